# round 4 V: conv_lite on eight waves with the DMA and MFMA roles split (tile 4,
# conv_lite_ws): numerics, per-layer time against conv_lite, ResNet-50 bench A/B
source tools/gpu_calls/gpu_steps.sh
step test_cpp 300 python -u -m pytest tests/test_conv_pp.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step probe 120 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3,s3_3x3s2 --impls lite,ws,lite,ws --reps 20
step bench_base 300 python -u bench.py --steps 20 --warmup 5
step bench_ws 300 env FT_CONV_LITE_WS=1 python -u bench.py --steps 20 --warmup 5
