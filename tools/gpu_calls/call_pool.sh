source tools/gpu_calls/gpu_steps.sh
step build 400 python -c "import __graft_entry__ as g; g.build()"
step pytest_k 300 python -m pytest tests/test_dconv.py tests/test_compiler.py -q -m gpu -x
step bench_resnet 500 python bench.py --steps 30 --warmup 5
cd /tmp && export TMPDIR=/tmp
step rocprof_rn 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rn2" -o run -- python "$REPO/bench.py" --steps 5 --warmup 2
