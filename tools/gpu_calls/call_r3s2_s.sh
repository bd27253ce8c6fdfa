# round 3 (session 2) R/S: conv_lite_fp8 channel tiles 128 / 96 / 64 (least Cout padding)
# and a single LDS stage for K <= 128; fp8 pool fusion only when the pooled tiling is tight
source tools/gpu_calls/gpu_steps.sh
step pytest_r 300 python -u -m pytest tests/test_fp8.py tests/test_dconv.py -m gpu -x -q --timeout 120 --timeout-method thread
step inc_static 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_static_b 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_dyn 500 python -u bench.py --model inception_v3 --steps 60 --warmup 10 --dynamic
step inc_layers 300 python -u bench/layer_table.py --model inception_v3
