# tail kernels with the next tile's residual prefetched during phase 2
source tools/gpu_calls/gpu_steps.sh
step tail_ab 120 python -u bench/tail_decimate_ab.py
step pytest_bn 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_bottleneck.py tests/test_fullsize_numerics.py
step layers 300 python -u bench/layer_table.py --model resnet50
step rn1 300 python -u bench.py --steps 40 --warmup 5
step rn2 300 python -u bench.py --steps 40 --warmup 5
