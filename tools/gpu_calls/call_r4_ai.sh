# round 4 AI: the 128x256 bf16 tile only where its grid keeps >= 768 workgroups
# (conv_lite_wide 2: ResNet-50's stage 3/4 expand + projection convs, Cout 1024 / 2048);
# plan-level numerics, then ResNet-50 A/B alternating on one box
source tools/gpu_calls/gpu_steps.sh
step test_plan 300 env FT_CONV_LITE_WIDE=2 python -u -m pytest tests/test_conv_pp.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step rn_base_a 300 python -u bench.py --steps 20 --warmup 5
step rn_w2_a 300 env FT_CONV_LITE_WIDE=2 python -u bench.py --steps 20 --warmup 5
step rn_base_b 300 python -u bench.py --steps 20 --warmup 5
step rn_w2_b 300 env FT_CONV_LITE_WIDE=2 python -u bench.py --steps 20 --warmup 5
step rn_base_c 300 python -u bench.py --steps 20 --warmup 5
step rn_w2_c 300 env FT_CONV_LITE_WIDE=2 python -u bench.py --steps 20 --warmup 5
