#!/bin/bash
# Round 6 call N: background JPEG decode in the runner (exactness, end to end), job-mode
# host phases against the SPMD bench.
source tools/gpu_calls/gpu_steps.sh
step r06_n/test_jpeg 300 python -u -m pytest tests/test_jpeg.py -x -v -m gpu --timeout 120 --timeout-method thread
step r06_n/jpeg_async32 400 python bench/jpeg_e2e.py --files 20000 --decode-threads 32
step r06_n/jpeg_async48 400 python bench/jpeg_e2e.py --files 20000 --decode-threads 48
step r06_n/bench_rn_job 300 python bench.py --job --steps 20 --warmup 5
step r06_n/bench_rn 200 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_n/bench_bert_job 300 python bench.py --model bert_graph --job --steps 30 --warmup 5
step r06_n/bench_bert 300 python bench.py --model bert_graph --steps 30 --warmup 5
