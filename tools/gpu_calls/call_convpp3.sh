# conv_pp selection timed with two concurrent lanes: A/B bench
source tools/gpu_calls/gpu_steps.sh
step bench_pp 300 python -u bench.py --steps 30 --warmup 5
FTM_CONV_IMPL=incumbent step bench_inc 300 python -u bench.py --steps 30 --warmup 5
step bench_pp2 300 python -u bench.py --steps 30 --warmup 5
FTM_CONV_IMPL=incumbent step bench_inc2 300 python -u bench.py --steps 30 --warmup 5
