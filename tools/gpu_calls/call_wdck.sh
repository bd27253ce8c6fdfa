# fused W&D checkpoint round trip
source tools/gpu_calls/gpu_steps.sh
step wd_ck 300 python -u -m pytest tests/test_widedeep.py -x -q -m gpu --timeout 250 --timeout-method thread
