# Persistent pooled stem: numerics (both kernels), A/B timing, end-to-end bench
source tools/gpu_calls/gpu_steps.sh
step pytest_dconv 300 python -u -m pytest tests/test_dconv.py -x -v -m gpu --timeout 120 --timeout-method thread
step stem 200 python bench/stem_ab.py 256
step bench_resnet 300 python bench.py --steps 40 --warmup 8
