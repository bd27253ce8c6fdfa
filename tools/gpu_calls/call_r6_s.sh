#!/bin/bash
# Round 6 call S: full GPU suite, smoke, and the headline bench on the current tree.
source tools/gpu_calls/gpu_steps.sh
step r06_s/pytest_gpu 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
step r06_s/smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r06_s/bench 200 python bench.py --gpus 1 --steps 20 --warmup 5
