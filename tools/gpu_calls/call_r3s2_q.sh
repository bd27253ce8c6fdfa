# round 3 (session 2) Q (rerun after the pooled fp8 template fix): fp8 direct conv + fused 3x3/s2 max pool (Inception Conv2d_2b ->
# MaxPool_3a); stream --processes re-measured
source tools/gpu_calls/gpu_steps.sh
step pytest_q 300 python -u -m pytest tests/test_dconv.py tests/test_fp8.py -m gpu -x -q --timeout 120 --timeout-method thread
step inc_static 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_static_b 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_dyn 500 python -u bench.py --model inception_v3 --steps 60 --warmup 10 --dynamic
step inc_layers 300 python -u bench/layer_table.py --model inception_v3
step stream_proc 300 python -u examples/resnet50_stream.py --records 200000 --processes
step stream_chain 300 python -u examples/resnet50_stream.py --records 200000
