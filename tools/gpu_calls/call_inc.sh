source tools/gpu_calls/gpu_steps.sh
step build 400 python -c "import __graft_entry__ as g; g.build()"
step pytest_fp8 300 python -m pytest tests/test_fp8.py -q -m gpu -x
step bench_inc_fp8 500 python bench.py --model inception_v3 --steps 20 --warmup 5
step bench_inc_dyn 500 python bench.py --model inception_v3 --steps 40 --warmup 5 --buckets 64,128 --dynamic
cd /tmp && export TMPDIR=/tmp
step rocprof_inc 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_inc2" -o run -- python "$REPO/bench.py" --model inception_v3 --steps 5 --warmup 2
