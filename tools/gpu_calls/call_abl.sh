source tools/gpu_calls/gpu_steps.sh
step build 400 python -c "import __graft_entry__ as g; g.build()"
step ablate 300 python bench/ablate_v2.py
