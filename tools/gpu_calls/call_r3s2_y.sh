# round 3 (session 2) Y: lane stagger A/B (lane 1 starts when lane 0's first batch is done:
# the two lanes run half a period apart instead of in step), ResNet-50 and Inception-v3
source tools/gpu_calls/gpu_steps.sh
step rn_base_a 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_stag_a 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --stagger-lanes
step rn_base_b 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_stag_b 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --stagger-lanes
step rn_base_300 300 python -u bench.py --gpus 1 --steps 300 --warmup 10
step rn_stag_300 300 python -u bench.py --gpus 1 --steps 300 --warmup 10 --stagger-lanes
step inc_base 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_stag 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --stagger-lanes
step inc_base_300 300 python -u bench.py --model inception_v3 --steps 300 --warmup 10
step inc_stag_300 300 python -u bench.py --model inception_v3 --steps 300 --warmup 10 --stagger-lanes
step inc_l3 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --lanes 3
