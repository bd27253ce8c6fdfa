# round 4 AA: the plan-level GPU tests of the opt-in DMA / MFMA-wave tiles
source tools/gpu_calls/gpu_steps.sh
step test_plans 300 python -u -m pytest tests/test_conv_pp.py::test_conv_lite_ws_in_resnet_plan_gpu tests/test_fp8.py::test_inception_v3_fp8_plan_gpu -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
