source tools/gpu_calls/gpu_steps.sh
step build 400 python -c "import __graft_entry__ as g; g.build()"
step pytest_k 300 python -m pytest tests/test_kernels_gpu.py tests/test_compiler.py -q -m gpu -x
step bench_resnet 500 python bench.py --steps 30 --warmup 5
step tune_bf16 300 python bench/conv_tune.py
