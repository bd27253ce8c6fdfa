# padding-free BERT: GPU tests, bench packed vs padded, profile of the packed encoder
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread
step bench_bert_pack 500 python bench.py --model bert --steps 30 --warmup 5
step bench_bert_pad 500 python bench.py --model bert --steps 30 --warmup 5 --no-pack
cd /tmp && export TMPDIR=/tmp
step rocprof_bert_pack 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bert_pack" -o run -- python "$REPO/bench.py" --model bert --steps 5 --warmup 2
