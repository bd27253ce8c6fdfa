#!/bin/bash
# Round 6 call AE: re-check the ResNet-50 plan switches against the new two-link chain default.
source tools/gpu_calls/gpu_steps.sh
step r06_ae/default_1 200 python bench.py --steps 20 --warmup 5
step r06_ae/no_pw_res 200 env FT_PW_RES_KERNEL=0 python bench.py --steps 20 --warmup 5
step r06_ae/no_c3x3c64 200 env FT_CONV3X3C64_KERNEL=0 python bench.py --steps 20 --warmup 5
step r06_ae/no_decimate 200 env FT_DECIMATE_TAILS=0 python bench.py --steps 20 --warmup 5
step r06_ae/default_2 200 python bench.py --steps 20 --warmup 5
step r06_ae/no_block_tails 200 env FT_FUSE_BLOCK_TAILS=0 python bench.py --steps 20 --warmup 5
step r06_ae/chain_batch64 200 env FT_CHAIN_BATCH=64 python bench.py --steps 20 --warmup 5
step r06_ae/default_3 200 python bench.py --steps 20 --warmup 5
