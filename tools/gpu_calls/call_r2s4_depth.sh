# ResNet-50: pipeline slots (depth) 2 vs 3 at 2 lanes — throughput and p50
source tools/gpu_calls/gpu_steps.sh
for i in 1 2; do
step d3_$i 300 python -u bench.py --steps 300 --warmup 10 --depth 3
step d2_$i 300 python -u bench.py --steps 300 --warmup 10 --depth 2
done
