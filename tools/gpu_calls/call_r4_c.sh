# round 4 C: conv_lite tile variants after the raw-s_barrier fix of the 3-stage loop (the
# __syncthreads of the first try drained the third stage): 4-wave 128x128 / 256x128 with
# 3 stages, and the new 8-wave 256x128 tile (2 waves per SIMD) with 3 / 2 stages, vs the
# default per layer; then the batch-slice chain (stage-1 intermediates per 16/32/64-image
# slice, resident in the Infinity Cache) and conv_lite for the stage-4 expands in the bench
source tools/gpu_calls/gpu_steps.sh
step test_conv 300 python -u -m pytest tests/test_conv_pp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
if ! grep -q " passed" "$OUT/test_conv.log" || grep -q "failed" "$OUT/test_conv.log"; then
  echo "[call] conv tests did not pass; no probes"; exit 1
fi
step probe_3x3 300 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3,s3_3x3s2 --impls lite,lites3,lite256s3,lite8s3,lite8 --reps 20
step probe_1x1 300 python -u bench/conv_layer_probe.py --layers s2_reduce,s3_reduce,s4_expand,s1_reduce --impls igemm,lite,lite8s3,lite8 --reps 20
step test_chain 300 python -u -m pytest tests/test_chain.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
if grep -q " passed" "$OUT/test_chain.log" && ! grep -q "failed" "$OUT/test_chain.log"; then
  step bench_default 300 python -u bench.py --steps 20 --warmup 5
  FT_CHAIN_BATCH=32 step bench_chain32 300 python -u bench.py --steps 20 --warmup 5
  FT_CHAIN_BATCH=64 step bench_chain64 300 python -u bench.py --steps 20 --warmup 5
  FT_CHAIN_BATCH=16 step bench_chain16 300 python -u bench.py --steps 20 --warmup 5
  FT_CHAIN_BATCH=32 FT_CHAIN_EDGE=1 step bench_chain32e 300 python -u bench.py --steps 20 --warmup 5
fi
FT_CONV_LITE_EXPAND=1 step bench_lite_expand 300 python -u bench.py --steps 20 --warmup 5
