# round 3 (session 2) H: conv_lite with a 32-deep K-tile (32 KiB LDS, igemm footprint):
# numerics, per-layer probe, ResNet-50 2-lane A/B against the incumbent igemm
source tools/gpu_calls/gpu_steps.sh
step pytest_convpp 300 python -u -m pytest tests/test_conv_pp.py -q -m gpu --timeout 120 --timeout-method thread
step probe 200 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3,s3_3x3s2 --impls igemm,lite,lite32 --reps 20
step rn_l32_a 200 env FT_CONV_LITE_BK=32 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_inc_a 200 env FT_CONV_IMPL=incumbent python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_l32_b 200 env FT_CONV_LITE_BK=32 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_inc_b 200 env FT_CONV_IMPL=incumbent python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_l32_s34 200 env FT_CONV_LITE_BK=32 FT_CONV_LITE_MAX_M=60000 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_l32_300 200 env FT_CONV_LITE_BK=32 python -u bench.py --gpus 1 --steps 300 --warmup 10
step rn_inc_300 200 env FT_CONV_IMPL=incumbent python -u bench.py --gpus 1 --steps 300 --warmup 10
