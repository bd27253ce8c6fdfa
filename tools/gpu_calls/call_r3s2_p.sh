# round 3 (session 2) P: Inception AvgPool -> 1x1 conv branches commuted (conv -> pool with
# bias/act/quantise epilogue), dynamic batching with a bucket every 8 and the in-flight cap;
# worker-operator chaining reverted (transport + stream --processes re-measured)
source tools/gpu_calls/gpu_steps.sh
step pytest_fp8 300 python -u -m pytest tests/test_fp8.py tests/test_arena.py -m gpu -x -q --timeout 120 --timeout-method thread
step inc_static 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_static_b 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_dyn 500 python -u bench.py --model inception_v3 --steps 60 --warmup 10 --dynamic
step inc_layers 300 python -u bench/layer_table.py --model inception_v3
step transport8 300 python -u bench/transport_bench.py --workers 8 --records 80000
step stream_proc 300 python -u examples/resnet50_stream.py --records 200000 --processes
step bench_rn 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
