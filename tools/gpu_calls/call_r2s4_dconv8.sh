# 8-wave (32 x 16 px) direct-conv tiles for the unpooled layers (Inception-v3 narrow convs)
source tools/gpu_calls/gpu_steps.sh
step pytest_dconv8 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_dconv.py tests/test_fp8.py
step dconv_tune 200 python -u bench/dconv_tune.py
for i in 1 2; do
step inc_w4_$i 300 env FTM_DCONV_WAVES=4 python -u bench.py --model inception_v3 --steps 100 --warmup 10
step inc_w8_$i 300 python -u bench.py --model inception_v3 --steps 100 --warmup 10
done
step rn_w8 300 python -u bench.py --steps 300 --warmup 10
