#!/bin/bash
# Round 6 call X: two-link vs three-link chain, interleaved three times.
source tools/gpu_calls/gpu_steps.sh
for i in 1 2 3; do
step r06_x/l2_$i 200 python bench.py --steps 20 --warmup 5
step r06_x/l3_$i 200 env FT_CHAIN_MAX_LINKS=3 python bench.py --steps 20 --warmup 5
done
