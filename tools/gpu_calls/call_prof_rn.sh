source tools/gpu_calls/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp
step rocprof_rn 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rn2" -o run -- python "$REPO/bench.py" --steps 5 --warmup 2
