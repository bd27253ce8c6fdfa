# round 3 (session 2) X: Inception sibling-conv fusion A/B on one box (EngineConfig
# sibling_conv_fusion), static and dynamic; the multi-output test with e4m3-subnormal slack
source tools/gpu_calls/gpu_steps.sh
step pytest_x 300 python -u -m pytest tests/test_fp8.py -m gpu -x -q --timeout 120 --timeout-method thread
step inc_on_a 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_off_a 300 env FT_SIBLING_CONV_FUSION=0 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_on_b 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_off_b 300 env FT_SIBLING_CONV_FUSION=0 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_on_300 300 python -u bench.py --model inception_v3 --steps 300 --warmup 10
step inc_off_300 300 env FT_SIBLING_CONV_FUSION=0 python -u bench.py --model inception_v3 --steps 300 --warmup 10
step inc_dyn_on 500 python -u bench.py --model inception_v3 --steps 60 --warmup 10 --dynamic
step inc_dyn_off 500 env FT_SIBLING_CONV_FUSION=0 python -u bench.py --model inception_v3 --steps 60 --warmup 10 --dynamic
