# round 4 H: conv_lite with the DMA split into prep (address VALU between the MFMA steps of
# the previous tile) and issue (8 bare LDS-DMA pieces after the barrier): correctness, the
# per-phase stamps, per-layer times, and the ResNet-50 bench (x2) / Inception-v3 (uses none)
source tools/gpu_calls/gpu_steps.sh
step test_conv 300 python -u -m pytest tests/test_conv_pp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
if ! grep -q " passed" "$OUT/test_conv.log" || grep -q "failed" "$OUT/test_conv.log"; then
  echo "[call] conv tests did not pass; no probes"; exit 1
fi
step stamp 120 python -u bench/conv_stamp_probe.py --layers s2_3x3,s3_3x3,s4_3x3
step probe_3x3 300 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3,s3_3x3s2 --impls lite --reps 20
step bench_rn_a 300 python -u bench.py --steps 20 --warmup 5
step bench_rn_b 300 python -u bench.py --steps 20 --warmup 5
step bench_rn_300 300 python -u bench.py --steps 300 --warmup 10
