source tools/gpu_calls/gpu_steps.sh
step build 400 python -c "import __graft_entry__ as g; g.build()"
step pytest_wd 300 python -m pytest tests/test_widedeep.py -q -m gpu
step bench_wd 300 python bench.py --model widedeep --steps 30 --warmup 5
cd /tmp && export TMPDIR=/tmp
step rocprof_wd 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_wd3" -o run -- python "$REPO/bench.py" --model widedeep --steps 5 --warmup 2
