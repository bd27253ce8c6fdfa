#!/bin/bash
# Round 6 call E: the recomputing stage-1 chain (tests, A/B bench), job modes with bulk
# sources, JPEG end to end, 8-rank host staging rehearsal.
source tools/gpu_calls/gpu_steps.sh
step r06_e/test_chain 300 python -u -m pytest tests/test_bottleneck.py -x -q -m gpu --timeout 120 --timeout-method thread
step r06_e/bench_rn_chain 200 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_e/bench_rn_nochain 200 env FT_RECOMPUTE_TAILS=0 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_e/bench_rn_chain2 200 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_e/bench_rn_nochain2 200 env FT_RECOMPUTE_TAILS=0 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_e/bench_rn_chain300 200 python bench.py --gpus 1 --steps 300 --warmup 10
step r06_e/bench_rn_job 300 python bench.py --job --steps 20 --warmup 5
step r06_e/bench_inc_job 300 python bench.py --model inception_v3 --job --steps 30 --warmup 5
step r06_e/bench_bert_job 300 python bench.py --model bert_graph --job --steps 30 --warmup 5
step r06_e/jpeg_e2e_r12 400 python bench/jpeg_e2e.py --files 20000 --readers 12
step r06_e/host_staging_8x2 120 python tools/host_staging_rehearsal.py --ranks 8 --threads 2 --seconds 6
step r06_e/host_staging_8x2_paced 120 python tools/host_staging_rehearsal.py --ranks 8 --threads 2 --seconds 6 --paced
