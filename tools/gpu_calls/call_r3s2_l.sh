# round 3 (session 2) L: in-process source chaining (source -> model operator on one thread)
# vs the unchained source thread, ResNet-50 stream at 200k records; plus the GPU suite
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step stream_chain 300 python -u examples/resnet50_stream.py --records 200000
step stream_nochain 300 python -u examples/resnet50_stream.py --records 200000 --no-chain
step stream_chain_sm 400 python -u examples/resnet50_stream.py --records 200000 --savedmodel
step stream_wsrc 300 python -u examples/resnet50_stream.py --records 200000 --worker-source
