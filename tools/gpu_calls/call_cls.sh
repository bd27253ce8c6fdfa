source tools/gpu_calls/gpu_steps.sh
step pytest_bert 300 python -u -m pytest tests/test_bert.py -x -v -m gpu --timeout 200 --timeout-method thread
step bench_bert 300 python bench.py --model bert --steps 30 --warmup 5
step bench_bert_l1 300 python bench.py --model bert --steps 30 --warmup 5 --lanes 1
