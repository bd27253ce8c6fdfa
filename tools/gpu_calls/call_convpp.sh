# conv_pp: numerics, then the ResNet layer micro-benchmark
source tools/gpu_calls/gpu_steps.sh
step pytest_convpp 300 python -u -m pytest tests/test_conv_pp.py -x -v -m gpu --timeout 120 --timeout-method thread
step bench_convpp 300 python -u bench/conv_pp_bench.py
