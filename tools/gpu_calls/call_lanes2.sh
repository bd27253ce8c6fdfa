source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread
step bench_rn_l2 300 python bench.py --steps 30 --warmup 5 --lanes 2
step bench_rn_l3 300 python bench.py --steps 30 --warmup 5 --lanes 3
step bench_rn_l4 300 python bench.py --steps 30 --warmup 5 --lanes 4
step bench_rn_l2_b128 300 python bench.py --steps 30 --warmup 5 --lanes 2 --batch 128
step bench_inc_l3 300 python bench.py --model inception_v3 --steps 20 --warmup 5 --lanes 3
step bench_bert_l4 300 python bench.py --model bert --steps 30 --warmup 5 --lanes 4
step bench_bert_pad_l3 300 python bench.py --model bert --steps 30 --warmup 5 --lanes 3 --no-pack
