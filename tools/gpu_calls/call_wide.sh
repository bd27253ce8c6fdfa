# Wide register-staged igemm tiles (cfg 5-8): numerics, then the ResNet layer sweep
source tools/gpu_calls/gpu_steps.sh
step pytest_conv 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "conv2d_nhwc or identity" --timeout 120 --timeout-method thread
step conv_tune 400 python bench/conv_tune.py 256
