source tools/gpu_calls/gpu_steps.sh
step rn_l2 200 python bench.py --steps 30 --warmup 5
step rn_l3 200 python bench.py --steps 30 --warmup 5 --lanes 3
step rn_l2_b384 200 python bench.py --steps 20 --warmup 5 --batch 384
step rn_l2_b512 200 python bench.py --steps 20 --warmup 5 --batch 512
step rn_l2_d4 200 python bench.py --steps 30 --warmup 5 --depth 4
step inc_l2 200 python bench.py --model inception_v3 --steps 30 --warmup 5
