# round 4 W: conv_lite_fp8 on DMA / MFMA waves (cfg 9, channel tiles <= 96) and the bf16
# conv_lite_ws: numerics, then Inception-v3 fp8 and ResNet-50 benches A/B (FT_CONV_LITE_WS);
# the batch-slice chain with a short last slice (dynamic batch sizes chain too)
source tools/gpu_calls/gpu_steps.sh
step test_ws 400 python -u -m pytest tests/test_fp8.py tests/test_conv_pp.py tests/test_chain.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step inc_base 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_ws 300 env FT_CONV_LITE_WS=1 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_base2 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_ws2 300 env FT_CONV_LITE_WS=1 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step rn_base 300 python -u bench.py --steps 20 --warmup 5
step rn_ws 300 env FT_CONV_LITE_WS=1 python -u bench.py --steps 20 --warmup 5
step inc_dyn 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
