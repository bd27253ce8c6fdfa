#!/bin/bash
# Round 6 call H: JPEG end to end with the decode deferred to the model's host stage
# (native decoder into the pinned slot), BERT job with staggered lanes, a cProfile of the
# ResNet job's worker chain against the SPMD bench on the same box.
source tools/gpu_calls/gpu_steps.sh
step r06_h/test_jpeg 200 python -u -m pytest tests/test_jpeg.py -x -q --timeout 120 --timeout-method thread
step r06_h/jpeg_e2e_staged16 400 python bench/jpeg_e2e.py --files 20000 --decode-threads 16
step r06_h/jpeg_e2e_staged32 400 python bench/jpeg_e2e.py --files 20000 --decode-threads 32
step r06_h/bench_bert_job 300 python bench.py --model bert_graph --job --steps 30 --warmup 5
step r06_h/bench_bert 300 python bench.py --model bert_graph --steps 30 --warmup 5
step r06_h/bench_rn 200 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_h/bench_rn_job 300 env FTM_WORKER_PROFILE="$OUT/r06_h/rnjob.prof" python bench.py --job --steps 20 --warmup 5
step r06_h/rnjob_pstats 60 python -c "
import glob, pstats, sys
for f in sorted(glob.glob('$OUT/r06_h/rnjob.prof.*')):
    print('==', f); pstats.Stats(f).sort_stats('tottime').print_stats(35); pstats.Stats(f).sort_stats('cumtime').print_stats(30)"
