# round 4 X: where the two-lane ResNet-50 bench's time goes when a kernel gets faster alone:
# one and three lanes, with and without the DMA / MFMA-wave conv_lite (tile 4)
source tools/gpu_calls/gpu_steps.sh
step rn_l1 300 python -u bench.py --steps 20 --warmup 5 --lanes 1
step rn_l1_ws 300 env FT_CONV_LITE_WS=1 python -u bench.py --steps 20 --warmup 5 --lanes 1
step rn_l3 300 python -u bench.py --steps 20 --warmup 5 --lanes 3
step rn_l3_ws 300 env FT_CONV_LITE_WS=1 python -u bench.py --steps 20 --warmup 5 --lanes 3
step rn_l2 300 python -u bench.py --steps 20 --warmup 5
