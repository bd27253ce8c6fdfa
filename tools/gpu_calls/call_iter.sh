source tools/gpu_calls/gpu_steps.sh
step build 300 python -c "import __graft_entry__ as g; g.build()"
step pytest_gpu 600 python -m pytest tests -q -m gpu
step bench 400 python bench.py --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python "$REPO/bench.py" --steps 10 --warmup 3
