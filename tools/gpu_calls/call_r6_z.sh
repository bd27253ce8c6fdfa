#!/bin/bash
# Round 6 call Z: the second lane's start offset at a pipeline restart (0 / 0.75 / 1.5 / 3 ms).
source tools/gpu_calls/gpu_steps.sh
for i in 1 2; do
for o in 0 750 1500 3000; do
step r06_z/off${o}_$i 200 python bench.py --steps 20 --warmup 5 --lane-offset-us $o
done
done
