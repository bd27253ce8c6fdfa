# full GPU suite + smoke after the W&D / activation / chaining changes
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
