# round 4 M: Inception-v3's chained stem replayed per H2D piece (one graph per 32-image
# slice right after that piece's preprocess, then the graph of the rest): chain tests,
# Inception benches (static x2, dynamic), and the fp8 / compiler GPU tests
source tools/gpu_calls/gpu_steps.sh
step test_m 400 python -u -m pytest tests/test_chain.py tests/test_fp8.py tests/test_compiler.py tests/test_fullsize_numerics.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread
if ! grep -q " passed" "$OUT/test_m.log" || grep -q "failed" "$OUT/test_m.log"; then
  echo "[call] tests did not pass; no benches"; exit 1
fi
step bench_inc_a 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step bench_inc_b 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step bench_inc_dyn 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
