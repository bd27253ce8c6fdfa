# round 3 (session 3) E: kernel stats of the BERT graph (packed) and Inception-v3 fp8 benches
source tools/gpu_calls/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step prof_bert 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bert" -o bert -- python3 bench.py --model bert_graph --steps 20 --warmup 5
step prof_inc 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_inc" -o inc -- python3 bench.py --model inception_v3 --steps 20 --warmup 5
step layers_inc 300 python -u bench/layer_table.py --model inception_v3
