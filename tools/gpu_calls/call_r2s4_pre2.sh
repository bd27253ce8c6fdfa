# row-staged s2d preprocess on unaligned (299 x 3 B) rows: numerics, timing, Inception-v3 end to end
source tools/gpu_calls/gpu_steps.sh
step pytest_pre2 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k preprocess
step pre_ab2 120 python -u bench/preprocess_ab.py
for i in 1 2; do
step incpix_$i 300 env FTM_PREPROCESS_PIXEL=1 python -u bench.py --model inception_v3 --steps 100 --warmup 10
step incrow_$i 300 python -u bench.py --model inception_v3 --steps 100 --warmup 10
done
