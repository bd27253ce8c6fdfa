#!/bin/bash
# Round 6 call AF: ResNet-50 with cache-resident batch slices (64 / 32 images) vs the default.
source tools/gpu_calls/gpu_steps.sh
for i in 1 2; do
step r06_af/default_$i 200 python bench.py --steps 20 --warmup 5
step r06_af/cb64_$i 200 env FT_CHAIN_BATCH=64 python bench.py --steps 20 --warmup 5
step r06_af/cb32_$i 200 env FT_CHAIN_BATCH=32 python bench.py --steps 20 --warmup 5
done
step r06_af/cb64_300 200 env FT_CHAIN_BATCH=64 python bench.py --steps 300 --warmup 10
step r06_af/default_300 200 python bench.py --steps 300 --warmup 10
