source tools/gpu_calls/gpu_steps.sh
step build 400 python -c "import __graft_entry__ as g; g.build()"
step pytest_gpu 900 python -m pytest tests -q -m gpu
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_resnet 500 python bench.py --steps 30 --warmup 5
step bench_inc_fp8 500 python bench.py --model inception_v3 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
step rocprof_inc 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_inc3" -o run -- python "$REPO/bench.py" --model inception_v3 --steps 5 --warmup 2
