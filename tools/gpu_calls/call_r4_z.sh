# round 4 Z: validation of the final tree on a fresh box — the whole GPU suite, smoke, the
# BASELINE benches in their default configuration, and a ResNet-50 kernel-stats profile
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_rn_a 300 python -u bench.py --steps 20 --warmup 5
step bench_rn_b 300 python -u bench.py --steps 20 --warmup 5
step bench_inc 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step bench_inc_dyn 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
step bench_bert_graph 300 python -u bench.py --model bert_graph --steps 30 --warmup 5
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
cd /tmp && export TMPDIR=/tmp
step rocprof_rn 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rn" -o run -- python "$REPO/bench.py" --steps 20 --warmup 3
