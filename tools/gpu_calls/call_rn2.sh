source tools/gpu_calls/gpu_steps.sh
step build 400 python -c "import __graft_entry__ as g; g.build()"
step bench_resnet_a 500 python bench.py --steps 30 --warmup 5
step bench_resnet_b 500 python bench.py --steps 60 --warmup 10
step bench_resnet_c 500 python bench.py --steps 30 --warmup 5
