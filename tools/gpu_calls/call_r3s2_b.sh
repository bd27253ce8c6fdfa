# round 3 (session 2) B: W&D (gemm_train + LDS radix sort) bench + kernel stats, launch check, packed BERT graph bench + stream
source tools/gpu_calls/gpu_steps.sh
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
step launch_check 120 python -u bench.py --gpus 2 --rehearse-fake-comm --launch-check
step bench_bert_graph 400 python -u bench.py --model bert_graph --steps 50 --warmup 5
step bert_stream 300 python -u examples/bert_stream.py --steady --records 16384
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step prof_wd 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_wd" -o wd -- python3 bench.py --model widedeep --steps 20 --warmup 5
