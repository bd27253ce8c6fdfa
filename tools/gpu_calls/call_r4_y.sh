# round 4 Y: lanes for Inception-v3 fp8 (static and dynamic batch sizes)
source tools/gpu_calls/gpu_steps.sh
step inc_dyn_l2 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
step inc_dyn_l3 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic --lanes 3
step inc_dyn_l4 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic --lanes 4
step inc_l3 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --lanes 3
step inc_l2 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
