#!/bin/bash
# Round 6 call V: the stage-1 chain limited to 2 links (the third tail reads y3 again)
# against 3 links and no chain: per-layer tables and interleaved benches.
source tools/gpu_calls/gpu_steps.sh
step r06_v/test_chain 300 env FT_CHAIN_MAX_LINKS=2 python -u -m pytest tests/test_bottleneck.py -x -q -m gpu --timeout 120 --timeout-method thread
step r06_v/layers_l2 300 env FT_CHAIN_MAX_LINKS=2 python -u tools/layer_table.py --model resnet50 --out gpurun_out/r06_v/layers_l2.md
step r06_v/bench_l3 200 python bench.py --steps 20 --warmup 5
step r06_v/bench_l2 200 env FT_CHAIN_MAX_LINKS=2 python bench.py --steps 20 --warmup 5
step r06_v/bench_off 200 env FT_RECOMPUTE_TAILS=0 python bench.py --steps 20 --warmup 5
step r06_v/bench_l3b 200 python bench.py --steps 20 --warmup 5
step r06_v/bench_l2b 200 env FT_CHAIN_MAX_LINKS=2 python bench.py --steps 20 --warmup 5
step r06_v/bench_offb 200 env FT_RECOMPUTE_TAILS=0 python bench.py --steps 20 --warmup 5
