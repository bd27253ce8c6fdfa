source tools/gpu_calls/gpu_steps.sh
step build 400 python -c "import __graft_entry__ as g; g.build()"
step pytest_gpu 600 python -m pytest tests -q -m gpu
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_wd 300 python bench.py --model widedeep --steps 30 --warmup 5
cd /tmp && export TMPDIR=/tmp
step rocprof_wd 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_wd" -o run -- python "$REPO/bench.py" --model widedeep --steps 5 --warmup 2
