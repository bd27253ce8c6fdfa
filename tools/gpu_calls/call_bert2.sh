source tools/gpu_calls/gpu_steps.sh
step build 400 python -c "import __graft_entry__ as g; g.build()"
step pytest_bert 300 python -m pytest tests/test_bert.py -q -m gpu
step bench_bert 500 python bench.py --model bert --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
step rocprof_bert 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bert2" -o run -- python "$REPO/bench.py" --model bert --steps 5 --warmup 2
