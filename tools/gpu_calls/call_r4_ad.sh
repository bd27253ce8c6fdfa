# round 4 AD: bf16 conv_lite on a 128x256 tile (tile 5, 32-deep K-tile; conv_lite_wide) for
# Cout >= 256 — the input tile staged once per 256 channels; numerics, per-layer times,
# ResNet-50 A/B alternating on one box
source tools/gpu_calls/gpu_steps.sh
step test_cpp 300 python -u -m pytest tests/test_conv_pp.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step probe 180 python -u bench/conv_layer_probe.py --layers s3_3x3,s4_3x3,s3_3x3s2,s3_reduce --impls lite,wide,lite,wide --reps 20
step rn_base_a 300 python -u bench.py --steps 20 --warmup 5
step rn_wide_a 300 env FT_CONV_LITE_WIDE=1 python -u bench.py --steps 20 --warmup 5
step rn_base_b 300 python -u bench.py --steps 20 --warmup 5
step rn_wide_b 300 env FT_CONV_LITE_WIDE=1 python -u bench.py --steps 20 --warmup 5
