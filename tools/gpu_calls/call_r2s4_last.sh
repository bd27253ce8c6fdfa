# final tree: GPU suite + smoke + headline bench
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu_last 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
step smoke_last 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_last 300 python -u bench.py
