#!/bin/bash
# Round 6 call L: where the JPEG job's time goes (runner host phases, cProfile of the
# model worker's source chain).
source tools/gpu_calls/gpu_steps.sh
step r06_l/jpeg_part32 400 python bench/jpeg_e2e.py --files 20000 --decode-threads 32
step r06_l/jpeg_prof 400 env FTM_WORKER_PROFILE="$OUT/r06_l/jpeg.prof" python bench/jpeg_e2e.py --files 20000 --decode-threads 32
step r06_l/jpeg_pstats 60 python -c "
import glob, os, pstats
for f in sorted(glob.glob('$OUT/r06_l/jpeg.prof.*'), key=os.path.getsize, reverse=True):
    print('==', f); pstats.Stats(f).sort_stats('tottime').print_stats(25); pstats.Stats(f).sort_stats('cumtime').print_stats(40)"
