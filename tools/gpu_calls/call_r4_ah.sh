# round 4 AH: conv_lite_fp8 tile chooser counted over whole waves of 512 workgroups
# (fp8_lite_wide 3: short 8x8 grids take narrower tiles) against the default (2)
source tools/gpu_calls/gpu_steps.sh
step test_fp8 400 python -u -m pytest tests/test_fp8.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step inc_w2_a 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_w3_a 300 env FT_FP8_LITE_WIDE=3 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_w2_b 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_w3_b 300 env FT_FP8_LITE_WIDE=3 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_w3_dyn 300 env FT_FP8_LITE_WIDE=3 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
step inc_w2_dyn 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
