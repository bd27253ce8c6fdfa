# round 4 AE: conv_lite_fp8 channel tile chosen to stage the fewest rows (cfg 11: 160 and 192
# wide tiles; Cout 320 / 448 / 288 no longer on 64- / 96-wide tiles) against cfg 10 (+192);
# numerics, Inception-v3 A/B alternating on one box
source tools/gpu_calls/gpu_steps.sh
step test_fp8 400 python -u -m pytest tests/test_fp8.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step inc_w1_a 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_w2_a 300 env FT_FP8_LITE_WIDE=2 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_w1_b 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_w2_b 300 env FT_FP8_LITE_WIDE=2 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_w2_dyn 300 env FT_FP8_LITE_WIDE=2 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
step inc_w1_dyn 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
