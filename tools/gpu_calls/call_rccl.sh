# direct RCCL binding on the device + the W&D trainer and GPU suites that touch comm
source tools/gpu_calls/gpu_steps.sh
step pytest_rccl 300 python -u -m pytest tests/test_rccl.py tests/test_dist.py tests/test_widedeep.py -x -v -m gpu --timeout 120 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
