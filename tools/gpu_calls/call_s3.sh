# Session-3 re-entry validation: tests, smoke, headline benches, per-layer ResNet trace
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_resnet 400 python bench.py --steps 30 --warmup 5
step bench_bert 400 python bench.py --model bert --steps 30 --warmup 5
cd /tmp && export TMPDIR=/tmp
step rocprof_rn 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_s3" -o run -- python "$REPO/bench.py" --steps 5 --warmup 2 --lanes 1
