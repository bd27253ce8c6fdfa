# round 4 P: stage-1 block tails (64-pixel variants) with two tiles' loads in flight
source tools/gpu_calls/gpu_steps.sh
step test_p 400 python -u -m pytest tests/test_bottleneck.py tests/test_compiler.py tests/test_fullsize_numerics.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread
if ! grep -q " passed" "$OUT/test_p.log" || grep -q "failed" "$OUT/test_p.log"; then
  echo "[call] tests did not pass; no benches"; exit 1
fi
step layers_rn 300 python -u tools/layer_table.py --reps 5 --out "$OUT/layers_rn.md"
step bench_rn_a 300 python -u bench.py --steps 20 --warmup 5
step bench_rn_b 300 python -u bench.py --steps 20 --warmup 5
step bench_rn_300 300 python -u bench.py --steps 300 --warmup 10
