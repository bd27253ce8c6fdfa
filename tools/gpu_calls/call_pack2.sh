source tools/gpu_calls/gpu_steps.sh
step pytest_bert 600 python -u -m pytest tests/test_bert.py -x -v -m gpu --timeout 300 --timeout-method thread
step bench_bert_pack 500 python bench.py --model bert --steps 30 --warmup 5
step bench_bert_pack_notab 500 env FTM_GEMM_TABLE=0 python bench.py --model bert --steps 30 --warmup 5
step bench_bert_pad 500 python bench.py --model bert --steps 30 --warmup 5 --no-pack
