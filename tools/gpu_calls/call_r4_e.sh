# round 4 E: Inception-v3 fp8 — conv_lite_fp8's eight-wave 256-pixel tile on three LDS
# stages (cfg 9) for the layers with enough workgroups, per layer and in the bench, and the
# stem (149x149 .. 71x71) run per 32-image slice with Infinity-Cache-resident intermediates
source tools/gpu_calls/gpu_steps.sh
step test_fp8 300 python -u -m pytest tests/test_fp8.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
if ! grep -q " passed" "$OUT/test_fp8.log" || grep -q "failed" "$OUT/test_fp8.log"; then
  echo "[call] fp8 tests did not pass; no benches"; exit 1
fi
step layers_inc 300 python -u tools/layer_table.py --model inception_v3 --reps 5 --out "$OUT/layers_inc.md"
FT_FP8_LITE_WIDE=256 step layers_inc_wide 300 python -u tools/layer_table.py --model inception_v3 --reps 5 --out "$OUT/layers_inc_wide.md"
step bench_inc 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
FT_FP8_LITE_WIDE=256 step bench_inc_wide256 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
FT_FP8_LITE_WIDE=128 step bench_inc_wide128 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
FT_CHAIN_BATCH=32 FT_CHAIN_MIN_HW=5041 FT_CHAIN_EDGE=1 step bench_inc_chain32 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
