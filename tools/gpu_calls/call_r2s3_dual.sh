# pw_dual (stage-2 entry expand + decimated projection on the persistent prefetching kernel)
source tools/gpu_calls/gpu_steps.sh
step pytest_sel 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pw_res.py tests/test_bottleneck.py tests/test_compiler.py tests/test_fullsize_numerics.py
step pw_bench 120 python -u bench/pw_res_bench.py
step ab_old1 300 env FTM_PW_DUAL=0 python -u bench.py --steps 40 --warmup 5
step ab_new1 300 python -u bench.py --steps 40 --warmup 5
step ab_old2 300 env FTM_PW_DUAL=0 python -u bench.py --steps 40 --warmup 5
step ab_new2 300 python -u bench.py --steps 40 --warmup 5
step layers 300 python -u bench/layer_table.py --model resnet50
