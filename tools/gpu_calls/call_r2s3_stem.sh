# persistent pooled stem + pw_res K-256 64-px tiles: numerics, per-layer, end-to-end A/B
source tools/gpu_calls/gpu_steps.sh
step pytest_sel 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dconv.py tests/test_pw_res.py tests/test_bottleneck.py tests/test_compiler.py tests/test_fullsize_numerics.py
step pw_bench 120 python -u bench/pw_res_bench.py
step layers_new 300 python -u bench/layer_table.py --model resnet50
step layers_old 300 env FTM_STEM_PERSIST=0 python -u bench/layer_table.py --model resnet50
step ab_old1 300 env FTM_STEM_PERSIST=0 python -u bench.py --steps 40 --warmup 5
step ab_new1 300 python -u bench.py --steps 40 --warmup 5
step ab_old2 300 env FTM_STEM_PERSIST=0 python -u bench.py --steps 40 --warmup 5
step ab_new2 300 python -u bench.py --steps 40 --warmup 5
