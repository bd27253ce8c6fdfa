# fp8 implicit GEMM: s_setprio around the MFMA clusters (FTM_FP8_PRIO) — tests, Inception-v3 end to end
source tools/gpu_calls/gpu_steps.sh
step pytest_fp8prio 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fp8.py tests/test_fullsize_numerics.py
for i in 1 2 3; do
step abf0_$i 300 env FTM_FP8_PRIO=0 python -u bench.py --model inception_v3 --steps 150 --warmup 10
step abf1_$i 300 python -u bench.py --model inception_v3 --steps 150 --warmup 10
done
step abf_dyn0 300 env FTM_FP8_PRIO=0 python -u bench.py --model inception_v3 --steps 50 --warmup 5 --dynamic
step abf_dyn1 300 python -u bench.py --model inception_v3 --steps 50 --warmup 5 --dynamic
