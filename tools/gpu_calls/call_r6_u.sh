#!/bin/bash
# Round 6 call U: Inception-v3 with and without the cache-resident batch slices of the stem
# (chain_batch auto = 32-image slices vs 0 = whole batch), bench and per-layer tables.
source tools/gpu_calls/gpu_steps.sh
step r06_u/inc_slices 300 python bench.py --model inception_v3 --steps 30 --warmup 5
step r06_u/inc_noslices 300 env FT_CHAIN_BATCH=0 python bench.py --model inception_v3 --steps 30 --warmup 5
step r06_u/inc_slices2 300 python bench.py --model inception_v3 --steps 30 --warmup 5
step r06_u/inc_noslices2 300 env FT_CHAIN_BATCH=0 python bench.py --model inception_v3 --steps 30 --warmup 5
step r06_u/inc_dyn_slices 300 python bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
step r06_u/inc_dyn_noslices 300 env FT_CHAIN_BATCH=0 python bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
step r06_u/layers_slices 300 python -u tools/layer_table.py --model inception_v3 --out gpurun_out/r06_u/layers_inc_slices.md
step r06_u/layers_noslices 300 env FT_CHAIN_BATCH=0 python -u tools/layer_table.py --model inception_v3 --out gpurun_out/r06_u/layers_inc_noslices.md
