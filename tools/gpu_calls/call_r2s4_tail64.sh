# stage-1 residual tail with 64-pixel tiles (104 KB LDS, FTM_TAIL_TP64) — tests, end to end
source tools/gpu_calls/gpu_steps.sh
step pytest_tail64 300 env FTM_TAIL_TP64=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_bottleneck.py tests/test_compiler.py tests/test_fullsize_numerics.py
for i in 1 2 3; do
step abt0_$i 300 python -u bench.py --steps 300 --warmup 10
step abt1_$i 300 env FTM_TAIL_TP64=1 python -u bench.py --steps 300 --warmup 10
done
