# round 5 C: Winograd kernel time from the kernel trace (no host overhead)
source tools/gpu_calls/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step wino_prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/wino_prof" -o wino -- python3 -u bench/wino_bench.py --reps 20
find "$OUT/wino_prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/wino_kernel_stats.csv" \;
