# round 3 (session 2) G: conv_lite in 2-lane vs 1-lane plans (ResNet-50), stage-3/4-only variant;
# conv_lite_fp8 numerics + Inception-v3 fp8 A/B
source tools/gpu_calls/gpu_steps.sh
step pytest_fp8 300 python -u -m pytest tests/test_fp8.py tests/test_compiler.py tests/test_conv_pp.py -q -m gpu --timeout 120 --timeout-method thread
step rn_inc 200 env FT_CONV_IMPL=incumbent python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_lite 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_lite_s34 200 env FT_CONV_LITE_MAX_M=60000 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_inc_l1 200 env FT_CONV_IMPL=incumbent python -u bench.py --gpus 1 --steps 20 --warmup 5 --lanes 1
step rn_lite_l1 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --lanes 1
step rn_inc2 200 env FT_CONV_IMPL=incumbent python -u bench.py --gpus 1 --steps 20 --warmup 5
step inc_inc 300 env FT_CONV_IMPL=incumbent python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_lite 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_lite_l1 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --lanes 1
step inc_inc_l1 300 env FT_CONV_IMPL=incumbent python -u bench.py --model inception_v3 --steps 30 --warmup 5 --lanes 1
step probe32 200 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3,s3_3x3s2 --impls igemm,lite,lite32 --reps 20
step rn_l32_a 200 env FT_CONV_LITE_BK=32 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_l32_b 200 env FT_CONV_LITE_BK=32 python -u bench.py --gpus 1 --steps 20 --warmup 5
