#!/bin/bash
# Round 6 call G: the LDS-DMA double-buffered stage-1 chain: exactness, per-layer times, A/B bench.
source tools/gpu_calls/gpu_steps.sh
step r06_g/test_chain 300 python -u -m pytest tests/test_bottleneck.py -x -q -m gpu --timeout 120 --timeout-method thread
step r06_g/layers_chain 300 python -u tools/layer_table.py --model resnet50 --out gpurun_out/r06_g/layers_chain.md
step r06_g/bench_rn_chain 200 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_g/bench_rn_nochain 200 env FT_RECOMPUTE_TAILS=0 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_g/bench_rn_chain2 200 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_g/bench_rn_nochain2 200 env FT_RECOMPUTE_TAILS=0 python bench.py --gpus 1 --steps 20 --warmup 5
