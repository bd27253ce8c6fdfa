# Re-entry validation: the full GPU suite, both headline benches
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step bench_rn 300 python -u bench.py --steps 30 --warmup 5
step bench_bert 300 python -u bench.py --model bert --steps 30 --warmup 5
