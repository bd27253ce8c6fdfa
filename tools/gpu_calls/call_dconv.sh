source tools/gpu_calls/gpu_steps.sh
step build 400 python -c "import __graft_entry__ as g; g.build()"
step pytest_dconv 300 python -m pytest tests/test_dconv.py -q -m gpu -x
step tune_dconv 300 python bench/dconv_tune.py
