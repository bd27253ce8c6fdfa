# round 5 D: Winograd with the conflict-aware LDS layout: numerics, per-layer A/B, kernel trace
source tools/gpu_calls/gpu_steps.sh
step test_wino 300 python -u -m pytest tests/test_wino.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step wino_bench 300 python -u bench/wino_bench.py
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step wino_prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/wino_prof_d" -o wino -- python3 -u bench/wino_bench.py --reps 20
python3 tools/rocpd_stats.py "$OUT"/wino_prof_d/wino_results.db "$OUT/wino_stats_d.csv"
python3 -c "import sys; sys.path.insert(0,'.'); from flink_tensorflow_amd import _ext; h=_ext.hip(required=True); print([ (H, h.wino_f23_layout(256,H,H)) for H in (56,28,14,7)])"
