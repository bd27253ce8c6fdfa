source tools/gpu_calls/gpu_steps.sh
step build 400 python -c "import __graft_entry__ as g; g.build()"
step pytest_k 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x
step gemm_tune 300 python bench/gemm_tune.py
