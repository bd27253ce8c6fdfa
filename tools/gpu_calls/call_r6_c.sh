#!/bin/bash
# Round 6 call C: GPU suite, Wide&Deep SPMD vs job mode, job modes of configs 2/3/5.
source tools/gpu_calls/gpu_steps.sh
step r06_c/pytest_gpu 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r06_c/bench_wd_spmd 200 python bench.py --model widedeep --steps 100 --warmup 10
step r06_c/bench_wd_job 300 python bench.py --model widedeep --job --steps 400 --warmup 20
step r06_c/bench_wd_job_spr16 300 python bench.py --model widedeep --job --steps 400 --warmup 20 --wd-steps-per-round 16
step r06_c/bench_inc 200 python bench.py --model inception_v3 --steps 30 --warmup 5
step r06_c/bench_inc_job 300 python bench.py --model inception_v3 --job --steps 30 --warmup 5
step r06_c/bench_bert 200 python bench.py --model bert_graph --steps 30 --warmup 5
step r06_c/bench_bert_job 300 python bench.py --model bert_graph --job --steps 30 --warmup 5
