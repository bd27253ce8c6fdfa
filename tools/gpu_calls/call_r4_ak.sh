# round 4 AK: the whole GPU suite and smoke on the final tree (fp8_lite_wide 2 default)
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_rn 300 python -u bench.py --steps 20 --warmup 5
