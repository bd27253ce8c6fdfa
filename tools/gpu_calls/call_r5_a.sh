# round 5 A: where the driver's 20-step window loses time (per-batch GPU timeline)
source tools/gpu_calls/gpu_steps.sh
step bench_tl1 300 python -u bench.py --steps 20 --warmup 5 --timeline
step bench_tl2 300 python -u bench.py --steps 20 --warmup 5 --timeline
step bench_300 300 python -u bench.py --steps 300 --warmup 5
