# round 4 AJ: steady-state rates of the final tree (300 steps) and the Inception-v3 fp8
# kernel mix on the wide channel tiles (rocprofv3 kernel stats)
source tools/gpu_calls/gpu_steps.sh
step rn_300 300 python -u bench.py --steps 300 --warmup 10
step inc_300 300 python -u bench.py --model inception_v3 --steps 300 --warmup 10
cd /tmp && export TMPDIR=/tmp
step rocprof_inc 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_inc" -o run -- python "$REPO/bench.py" --model inception_v3 --steps 20 --warmup 3
