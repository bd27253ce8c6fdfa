#!/bin/bash
# Round 6 call J: the two-wave conv_lite tile (128 x 64 outputs per wave): exactness,
# per-layer times and the A/B bench against the four-wave tile.
source tools/gpu_calls/gpu_steps.sh
step r06_j/test_conv_pp 300 python -u -m pytest tests/test_conv_pp.py -x -q -m gpu --timeout 120 --timeout-method thread
step r06_j/layers_w2 300 env FT_CONV_LITE_WAVES=2 python -u tools/layer_table.py --model resnet50 --out gpurun_out/r06_j/layers_w2.md
step r06_j/layers_w4 300 python -u tools/layer_table.py --model resnet50 --out gpurun_out/r06_j/layers_w4.md
step r06_j/bench_w2 200 env FT_CONV_LITE_WAVES=2 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_j/bench_w4 200 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_j/bench_w2b 200 env FT_CONV_LITE_WAVES=2 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_j/bench_w4b 200 python bench.py --gpus 1 --steps 20 --warmup 5
