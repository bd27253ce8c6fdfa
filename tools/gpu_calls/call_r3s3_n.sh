# round 3 (session 3) N: compute lanes 2 vs 3 under the lanes+1 in-flight cap
# (Inception-v3 fp8 and ResNet-50; throughput and p50)
source tools/gpu_calls/gpu_steps.sh
for i in a b; do
  step inc_l2_$i 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
  step inc_l3_$i 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --lanes 3
done
step inc_l2_300 300 python -u bench.py --model inception_v3 --steps 300 --warmup 10
step inc_l3_300 300 python -u bench.py --model inception_v3 --steps 300 --warmup 10 --lanes 3
step rn_l2_a 300 python -u bench.py --steps 20 --warmup 5
step rn_l3_a 300 python -u bench.py --steps 20 --warmup 5 --lanes 3
step rn_l2_300 300 python -u bench.py --steps 300 --warmup 10
step rn_l3_300 300 python -u bench.py --steps 300 --warmup 10 --lanes 3
