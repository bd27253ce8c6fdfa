# round 3 (session 2) F: conv_lite on the compiled ResNet-50 / Inception paths — numerics tests,
# bench A/B against the incumbent igemm (20-step window x2 each, 300 steps), kernel stats
source tools/gpu_calls/gpu_steps.sh
step pytest_num 600 python -u -m pytest tests/test_fullsize_numerics.py tests/test_compiler.py tests/test_model_function_compiled.py tests/test_conv_pp.py -q -m gpu --timeout 300 --timeout-method thread
step rn_lite_a 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_inc_a 200 env FT_CONV_IMPL=incumbent python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_lite_b 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_inc_b 200 env FT_CONV_IMPL=incumbent python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_lite_300 200 python -u bench.py --gpus 1 --steps 300 --warmup 10
step rn_lite_nopw 200 env FT_CONV_LITE_POINTWISE=0 python -u bench.py --gpus 1 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step prof_rn 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rn_lite" -o rn -- python3 bench.py --gpus 1 --steps 20 --warmup 5
