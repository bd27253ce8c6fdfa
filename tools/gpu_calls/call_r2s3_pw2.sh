# pw_res tile variants (K 256 tp 64, K 512 64x64) + gemm_pp for the K-512 stage-3 entry reduce
source tools/gpu_calls/gpu_steps.sh
step pytest_pw 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_pw_res.py
step pw_bench 120 python -u bench/pw_res_bench.py
step pytest_sel 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_bottleneck.py tests/test_compiler.py tests/test_fullsize_numerics.py
step ab_old1 300 env FTM_PP_MIN_K=1024 python -u bench.py --steps 40 --warmup 5
step ab_new1 300 python -u bench.py --steps 40 --warmup 5
step ab_old2 300 env FTM_PP_MIN_K=1024 python -u bench.py --steps 40 --warmup 5
step ab_new2 300 python -u bench.py --steps 40 --warmup 5
step layers 300 python -u bench/layer_table.py --model resnet50
