# s_setprio around the MFMA clusters of conv3x3c64 / pw_res / dconv (FTM_MFMA_PRIO) — tests, end to end
source tools/gpu_calls/gpu_steps.sh
step pytest_prio2 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dconv.py tests/test_pw_res.py tests/test_bottleneck.py tests/test_compiler.py
for i in 1 2 3; do
step abm0_$i 300 env FTM_MFMA_PRIO=0 python -u bench.py --steps 300 --warmup 10
step abm1_$i 300 python -u bench.py --steps 300 --warmup 10
done
step incm0 300 env FTM_MFMA_PRIO=0 python -u bench.py --model inception_v3 --steps 100 --warmup 10
step incm1 300 python -u bench.py --model inception_v3 --steps 100 --warmup 10
