# round 3 (session 3) G: GPU-only replay rate of the ResNet-50 plans (input resident in HBM,
# no host staging) on 1/2/3 lanes, next to bench.py in the same call
source tools/gpu_calls/gpu_steps.sh
step gpu_only 300 python -u bench/gpu_only_probe.py --lanes 1,2,3 --iters 300
step bench_300 300 python -u bench.py --steps 300 --warmup 10
step gpu_only_b 300 python -u bench/gpu_only_probe.py --lanes 2,1 --iters 300
