# round 4 R: conv_lite_fp8 K walk from an LDS table (one ds_read_b64 per lane and K-tile
# instead of the per-lane divmod walk): fp8 tests, K-tile phases, per-layer times, Inception bench
source tools/gpu_calls/gpu_steps.sh
step test_fp8 400 python -u -m pytest tests/test_fp8.py tests/test_fullsize_numerics.py tests/test_chain.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step stamp_fp8 120 python -u bench/conv_stamp_probe.py --fp8
step bench_inc1 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step bench_inc2 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step bench_incdyn 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
