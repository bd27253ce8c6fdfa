# round 4 E: Inception-v3 fp8 with the stem (149x149 .. 71x71, ~0.35-0.7 GB per 256-image
# tensor) run per image slice, repeated against the default on the same box; its per-layer
# table (per-step time summed over the slices)
source tools/gpu_calls/gpu_steps.sh
step inc_default_a 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
FT_CHAIN_BATCH=32 FT_CHAIN_MIN_HW=5041 FT_CHAIN_EDGE=1 step inc_chain32_a 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_default_b 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
FT_CHAIN_BATCH=32 FT_CHAIN_MIN_HW=5041 FT_CHAIN_EDGE=1 step inc_chain32_b 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
FT_CHAIN_BATCH=64 FT_CHAIN_MIN_HW=5041 FT_CHAIN_EDGE=1 step inc_chain64 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
FT_CHAIN_BATCH=16 FT_CHAIN_MIN_HW=5041 FT_CHAIN_EDGE=1 step inc_chain16 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
FT_CHAIN_BATCH=32 FT_CHAIN_MIN_HW=5041 step inc_chain32_noedge 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
FT_CHAIN_BATCH=32 FT_CHAIN_MIN_HW=5041 FT_CHAIN_EDGE=1 step inc_chain32_dyn 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
FT_CHAIN_BATCH=32 FT_CHAIN_MIN_HW=5041 FT_CHAIN_EDGE=1 step layers_inc_chain32 300 python -u tools/layer_table.py --model inception_v3 --reps 5 --out "$OUT/layers_inc_chain32.md"
