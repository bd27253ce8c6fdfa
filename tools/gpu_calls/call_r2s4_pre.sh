# row-staged s2d preprocess kernel: numerics vs the per-pixel kernel + host path, timing, end to end
source tools/gpu_calls/gpu_steps.sh
step pytest_pre 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k preprocess
step pre_ab 120 python -u bench/preprocess_ab.py
for i in 1 2; do
step abpix_$i 300 env FTM_PREPROCESS_PIXEL=1 python -u bench.py --steps 300 --warmup 10
step abrow_$i 300 python -u bench.py --steps 300 --warmup 10
done
