source tools/gpu_steps.sh
step build 400 python -c "import __graft_entry__ as g; g.build()"
step pytest_gpu 600 python -m pytest tests -q -m gpu -x
step tune 600 python bench/conv_tune.py 256
step bench 400 python bench.py --steps 20 --warmup 5
