# ResNet-50 operating point re-check with the igemm MFMA priority: 2 vs 3 compute lanes (depth 3 / 4)
source tools/gpu_calls/gpu_steps.sh
for i in 1 2; do
step l2_$i 300 python -u bench.py --steps 300 --warmup 10 --lanes 2
step l3_$i 300 python -u bench.py --steps 300 --warmup 10 --lanes 3
step l3d4_$i 300 python -u bench.py --steps 300 --warmup 10 --lanes 3 --depth 4
done
