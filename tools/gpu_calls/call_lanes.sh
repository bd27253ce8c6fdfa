source tools/gpu_calls/gpu_steps.sh
step pytest_lanes 300 python -u -m pytest tests/test_arena.py tests/test_remote.py -x -v -m gpu --timeout 200 --timeout-method thread
step bench_bert_l1 300 python bench.py --model bert --steps 30 --warmup 5 --lanes 1
step bench_bert_l2 300 python bench.py --model bert --steps 30 --warmup 5 --lanes 2
step bench_bert_l3 300 python bench.py --model bert --steps 30 --warmup 5 --lanes 3
step bench_rn_l1 300 python bench.py --steps 30 --warmup 5 --lanes 1
step bench_rn_l2 300 python bench.py --steps 30 --warmup 5 --lanes 2
step bench_inc_l2 300 python bench.py --model inception_v3 --steps 20 --warmup 5 --lanes 2
step bench_inc_l1 300 python bench.py --model inception_v3 --steps 20 --warmup 5 --lanes 1
