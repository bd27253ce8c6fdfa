# round 3 (session 2) N: framework-owned streams, step by step (the GPU suite segfaulted in
# the first runner test after utils/streams.py: a destroyed stream was still named by the
# pinned-host allocator; streams now go to a free list instead)
source tools/gpu_calls/gpu_steps.sh
step runner_probe 120 python -u tools/probes/runner_probe.py
step pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_rn 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_bert 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --model bert_graph
step stream_chain 300 python -u examples/resnet50_stream.py --records 200000
