#!/bin/bash
# Round 6 call AK: Inception-v3 (3 lanes) lane start offset 0 / 750 / 1500 us.
source tools/gpu_calls/gpu_steps.sh
for i in 1 2; do
for o in 0 750 1500; do
step r06_ak/inc_off${o}_$i 300 python bench.py --model inception_v3 --steps 30 --warmup 5 --lane-offset-us $o
done
done
