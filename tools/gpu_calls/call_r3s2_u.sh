# round 3 (session 2) U: ResNet expand + projection shortcut on the two-source conv_lite
# (DUAL) instead of the register-staged dual igemm; A/B against FT_CONV_IMPL=incumbent
source tools/gpu_calls/gpu_steps.sh
step pytest_u 400 python -u -m pytest tests/test_conv_pp.py tests/test_compiler.py tests/test_bottleneck.py tests/test_fullsize_numerics.py -m gpu -x -q --timeout 120 --timeout-method thread
step rn_a 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_inc 200 env FT_CONV_IMPL=incumbent python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_b 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_300 300 python -u bench.py --gpus 1 --steps 300 --warmup 10
step rn_layers 300 python -u bench/layer_table.py --model resnet50
