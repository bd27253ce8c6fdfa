# Arena validation: GPU tests touching compiled plans, smoke, resnet + inception bench
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_resnet 500 python bench.py --steps 30 --warmup 5
step bench_inc_dyn 500 python bench.py --model inception_v3 --steps 20 --warmup 5 --buckets 64,128 --dynamic
