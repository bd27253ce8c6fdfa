#!/bin/bash
# Round 6 call F: per-layer times of the recomputing stage-1 chain (on / off) and rocprof
# kernel stats of the two-lane bench with and without it.
source tools/gpu_calls/gpu_steps.sh
step r06_f/layers_chain 300 python -u tools/layer_table.py --model resnet50 --out gpurun_out/r06_f/layers_chain.md
step r06_f/layers_nochain 300 env FT_RECOMPUTE_TAILS=0 python -u tools/layer_table.py --model resnet50 --out gpurun_out/r06_f/layers_nochain.md
cd /tmp && export TMPDIR=/tmp
step r06_f/prof_chain 300 rocprofv3 --kernel-trace --stats -d "$OUT/r06_f/prof_chain" -o run -- python "$REPO/bench.py" --steps 20 --warmup 5
step r06_f/prof_nochain 300 env FT_RECOMPUTE_TAILS=0 rocprofv3 --kernel-trace --stats -d "$OUT/r06_f/prof_nochain" -o run -- python "$REPO/bench.py" --steps 20 --warmup 5
