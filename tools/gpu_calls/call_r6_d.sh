#!/bin/bash
# Round 6 call D: job modes with bulk sources, JPEG end to end, 8-rank host staging rehearsal.
source tools/gpu_calls/gpu_steps.sh
step r06_d/bench_rn 200 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_d/bench_rn_job 300 python bench.py --job --steps 20 --warmup 5
step r06_d/bench_inc 200 python bench.py --model inception_v3 --steps 30 --warmup 5
step r06_d/bench_inc_job 300 python bench.py --model inception_v3 --job --steps 30 --warmup 5
step r06_d/bench_bert 200 python bench.py --model bert_graph --steps 30 --warmup 5
step r06_d/bench_bert_job 300 python bench.py --model bert_graph --job --steps 30 --warmup 5
step r06_d/jpeg_e2e_r12 400 python bench/jpeg_e2e.py --files 20000 --readers 12
step r06_d/host_staging_8x2 120 python tools/host_staging_rehearsal.py --ranks 8 --threads 2 --seconds 6
step r06_d/host_staging_8x2_paced 120 python tools/host_staging_rehearsal.py --ranks 8 --threads 2 --seconds 6 --paced
step r06_d/host_staging_8x8 120 python tools/host_staging_rehearsal.py --ranks 8 --threads 8 --seconds 6
