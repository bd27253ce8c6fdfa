#!/bin/bash
# Round 6 call I: job workers NUMA-bound to their GPU (ResNet / Inception / BERT jobs vs
# SPMD), cProfile of the JPEG job's model worker.
source tools/gpu_calls/gpu_steps.sh
step r06_i/bench_rn_job 300 python bench.py --job --steps 20 --warmup 5
step r06_i/bench_rn 200 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_i/bench_rn_job2 300 python bench.py --job --steps 20 --warmup 5
step r06_i/bench_inc_job 300 python bench.py --model inception_v3 --job --steps 30 --warmup 5
step r06_i/bench_inc 300 python bench.py --model inception_v3 --steps 30 --warmup 5
step r06_i/bench_bert_job 300 python bench.py --model bert_graph --job --steps 30 --warmup 5
step r06_i/jpeg_e2e_bulk 400 python bench/jpeg_e2e.py --files 20000 --decode-threads 32
step r06_i/jpeg_e2e_prof 400 env FTM_WORKER_PROFILE="$OUT/r06_i/jpeg.prof" python bench/jpeg_e2e.py --files 20000 --decode-threads 32
step r06_i/jpeg_pstats 60 python -c "
import glob, pstats
for f in sorted(glob.glob('$OUT/r06_i/jpeg.prof.*')):
    print('==', f); pstats.Stats(f).sort_stats('tottime').print_stats(30); pstats.Stats(f).sort_stats('cumtime').print_stats(40)"
