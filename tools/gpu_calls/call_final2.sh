# round-2 final: GPU suite, every bench config, kernel-stat profiles of the four bench models
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_resnet 300 python -u bench.py --steps 30 --warmup 5
step bench_bert 300 python -u bench.py --model bert --steps 30 --warmup 5
step bench_bert_graph 300 python -u bench.py --model bert_graph --steps 30 --warmup 5
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
step bench_inc 300 python -u bench.py --model inception_v3 --steps 20 --warmup 5
step bench_inc_dyn 300 python -u bench.py --model inception_v3 --steps 20 --warmup 5 --dynamic
cd /tmp && export TMPDIR=/tmp
step prof_rn 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rn" -o run -- python "$REPO/bench.py" --steps 10 --warmup 3
step prof_bert 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bert" -o run -- python "$REPO/bench.py" --model bert --steps 10 --warmup 3
step prof_inc 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_inc" -o run -- python "$REPO/bench.py" --model inception_v3 --steps 10 --warmup 3
step prof_wd 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_wd" -o run -- python "$REPO/bench.py" --model widedeep --steps 20 --warmup 5
