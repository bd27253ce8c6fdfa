source tools/gpu_calls/gpu_steps.sh
step build 400 python -c "import __graft_entry__ as g; g.build()"
step pytest_v2 300 python -m pytest tests/test_kernels_gpu.py tests/test_fp8.py -q -m gpu -x
step tune_bf16 300 python bench/conv_tune.py
step tune_fp8 300 python bench/conv_tune_fp8.py
