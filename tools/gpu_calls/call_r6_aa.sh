#!/bin/bash
# Round 6 call AA: cProfile of the JPEG job's worker (Inception-v3, 299x299 files).
source tools/gpu_calls/gpu_steps.sh
step r06_aa/jpeg_inc_prof 500 env FTM_WORKER_PROFILE="$OUT/r06_aa/inc.prof" python bench/jpeg_e2e.py --files 20000 --model inception_v3
step r06_aa/pstats 60 python -c "
import glob, os, pstats
for f in sorted(glob.glob('$OUT/r06_aa/inc.prof.*'), key=os.path.getsize, reverse=True)[:1]:
    print('==', f); pstats.Stats(f).sort_stats('tottime').print_stats(30); pstats.Stats(f).sort_stats('cumtime').print_stats(45)"
