# Divide-free conv K walk + buffer-descriptor loads in igemm_bf16: numerics, layer sweep, bench
source tools/gpu_calls/gpu_steps.sh
step pytest_k 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_compiler.py tests/test_bottleneck.py -x -q -m gpu --timeout 120 --timeout-method thread
step conv_tune 400 python bench/conv_tune.py 256
step bench_resnet 300 python bench.py --steps 40 --warmup 8
