#!/bin/bash
# Round 6 call AG: Inception-v3 pipeline depth (slots) 3 / 4 / 6 on three lanes.
source tools/gpu_calls/gpu_steps.sh
for i in 1 2; do
step r06_ag/d3_$i 300 python bench.py --model inception_v3 --steps 30 --warmup 5
step r06_ag/d4_$i 300 python bench.py --model inception_v3 --steps 30 --warmup 5 --depth 4
step r06_ag/d6_$i 300 python bench.py --model inception_v3 --steps 30 --warmup 5 --depth 6
done
