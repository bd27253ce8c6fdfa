# ResNet-50 operating points with / without conv_pp
source tools/gpu_calls/gpu_steps.sh
step op_l2_inc 300 python -u bench.py --steps 30 --warmup 5
FTM_CONV_IMPL=pp step op_l2_pp 300 python -u bench.py --steps 30 --warmup 5
FTM_CONV_IMPL=auto step op_l1_b512_auto 300 python -u bench.py --steps 20 --warmup 5 --lanes 1 --batch 512
step op_l1_b512_inc 300 python -u bench.py --steps 20 --warmup 5 --lanes 1 --batch 512
step op_l3_inc 300 python -u bench.py --steps 30 --warmup 5 --lanes 3
FTM_CONV_IMPL=auto step op_l1_auto 300 python -u bench.py --steps 30 --warmup 5 --lanes 1
step op_l1_inc 300 python -u bench.py --steps 30 --warmup 5 --lanes 1
