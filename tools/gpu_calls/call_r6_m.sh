#!/bin/bash
# Round 6 call M: conv_lite with deeper DMA prefetch (tile 7: 32-deep K-tiles on 4 stages;
# tile 9: 64-deep on 3 stages): exactness, per-layer probe, A/B bench.
source tools/gpu_calls/gpu_steps.sh
step r06_m/test_conv_pp 300 python -u -m pytest tests/test_conv_pp.py -x -q -m gpu --timeout 120 --timeout-method thread
step r06_m/probe 200 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3 --impls lite:2,lite:7,lite:8,lite:9,lite:4 --reps 20
step r06_m/bench_t7 200 env FT_CONV_LITE_TILE=7 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_m/bench_t2 200 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_m/bench_t9 200 env FT_CONV_LITE_TILE=9 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_m/bench_t7b 200 env FT_CONV_LITE_TILE=7 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_m/bench_t2b 200 python bench.py --gpus 1 --steps 20 --warmup 5
