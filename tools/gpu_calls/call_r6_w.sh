#!/bin/bash
# Round 6 call W: the two-link chain default: exactness tests, full-size numerics, bench.
source tools/gpu_calls/gpu_steps.sh
step r06_w/tests 500 python -u -m pytest tests/test_bottleneck.py tests/test_compiler.py tests/test_fullsize_numerics.py -q -m gpu --timeout 120 --timeout-method thread
step r06_w/bench1 200 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_w/bench2 200 python bench.py --gpus 1 --steps 20 --warmup 5
step r06_w/bench300 200 python bench.py --gpus 1 --steps 300 --warmup 10
step r06_w/layers 300 python -u tools/layer_table.py --model resnet50 --out gpurun_out/r06_w/layers_rn.md
