source tools/gpu_calls/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp
step rocprof_rn 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rn_l2" -o run -- python "$REPO/bench.py" --steps 10 --warmup 3
step rocprof_bert 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bert_l3" -o run -- python "$REPO/bench.py" --model bert --steps 10 --warmup 3
step rocprof_inc 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_inc_l2" -o run -- python "$REPO/bench.py" --model inception_v3 --steps 10 --warmup 3
