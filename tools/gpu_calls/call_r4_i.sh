# round 4 I: the unrolled 3x3 fp8 max pool (all window loads issued before the first use):
# correctness, Inception-v3 per-layer table (stem chained, as the default plan runs) and
# the Inception bench x2
source tools/gpu_calls/gpu_steps.sh
step test_fp8 300 python -u -m pytest tests/test_fp8.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
if ! grep -q " passed" "$OUT/test_fp8.log" || grep -q "failed" "$OUT/test_fp8.log"; then
  echo "[call] fp8 tests did not pass; no benches"; exit 1
fi
step layers_inc 300 python -u tools/layer_table.py --model inception_v3 --reps 5 --out "$OUT/layers_inc.md"
step bench_inc_a 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step bench_inc_b 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step bench_inc_dyn 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
