# round 4 AL: the rebuilt kernel library (tile-choice binding added) — fp8 tests and smoke
source tools/gpu_calls/gpu_steps.sh
step test_fp8 400 python -u -m pytest tests/test_fp8.py -x -q -m "gpu or not gpu" -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
