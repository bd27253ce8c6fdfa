#!/bin/bash
# Round 6 call AH: rocprofv3 kernel statistics of the final ResNet-50 and Inception-v3 benches.
source tools/gpu_calls/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp
step r06_ah/prof_rn 300 rocprofv3 --kernel-trace --stats -d "$OUT/r06_ah/prof_rn" -o run -- python "$REPO/bench.py" --steps 20 --warmup 5
step r06_ah/prof_inc 300 rocprofv3 --kernel-trace --stats -d "$OUT/r06_ah/prof_inc" -o run -- python "$REPO/bench.py" --model inception_v3 --steps 30 --warmup 5
