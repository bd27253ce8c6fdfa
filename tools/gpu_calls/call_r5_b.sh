# round 5 B: Winograd F(2x2,3x3) kernel numerics + per-layer A/B
source tools/gpu_calls/gpu_steps.sh
step test_wino 300 python -u -m pytest tests/test_wino.py -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step wino_bench 300 python -u bench/wino_bench.py
