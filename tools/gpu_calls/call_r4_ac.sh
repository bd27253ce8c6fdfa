# round 4 AC: conv_lite_fp8 with a 192-wide channel tile (cfg 10, fp8_lite_wide): one tile
# of 192 channels stages 40 KiB per K-tile where two 96-wide tiles stage 56 KiB; numerics,
# then Inception-v3 A/B alternating on one box
source tools/gpu_calls/gpu_steps.sh
step test_fp8 400 python -u -m pytest tests/test_fp8.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step inc_base_a 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_wide_a 300 env FT_FP8_LITE_WIDE=1 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_base_b 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_wide_b 300 env FT_FP8_LITE_WIDE=1 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_wide_dyn 300 env FT_FP8_LITE_WIDE=1 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
step inc_base_dyn 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
