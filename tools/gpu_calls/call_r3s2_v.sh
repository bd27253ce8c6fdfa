# round 3 (session 2) V: Inception module heads (sibling 1x1 convs + the commuted pool
# branch) as one multi-output conv_lite_fp8 GEMM
source tools/gpu_calls/gpu_steps.sh
step pytest_v 300 python -u -m pytest tests/test_fp8.py -m gpu -x -q --timeout 120 --timeout-method thread
step inc_static 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_static_b 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_dyn 500 python -u bench.py --model inception_v3 --steps 60 --warmup 10 --dynamic
step inc_layers 300 python -u bench/layer_table.py --model inception_v3
step inc_numerics 300 python -u -m pytest tests/test_fullsize_numerics.py -m gpu -x -q -k inception --timeout 200 --timeout-method thread
