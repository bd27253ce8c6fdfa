# round 5 F: Winograd numerics + ablations (1: no bf16->f16 convert, 2: no MFMA)
source tools/gpu_calls/gpu_steps.sh
step test_wino 300 python -u -m pytest tests/test_wino.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step wino_bench 300 python -u bench/wino_bench.py
export FTM_WINO_DBG=1; step wino_dbg1 300 python -u bench/wino_bench.py --wino-only
export FTM_WINO_DBG=2; step wino_dbg2 300 python -u bench/wino_bench.py --wino-only
