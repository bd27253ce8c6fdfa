source tools/gpu_calls/gpu_steps.sh
step bench_bert 300 python bench.py --model bert --steps 30 --warmup 5
step bench_rn 300 python bench.py --steps 30 --warmup 5
step bench_inc 300 python bench.py --model inception_v3 --steps 30 --warmup 5
