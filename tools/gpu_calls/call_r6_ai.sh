#!/bin/bash
# Round 6 call AI: ResNet-50 job vs SPMD on the final tree (two-link chain), twice.
source tools/gpu_calls/gpu_steps.sh
for i in 1 2; do
step r06_ai/rn_$i 200 python bench.py --steps 20 --warmup 5
step r06_ai/rn_job_$i 300 python bench.py --job --steps 20 --warmup 5
done
