# Round-end check of the committed tree: GPU tests + smoke
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
