source tools/gpu_calls/gpu_steps.sh
step build 400 python -c "import __graft_entry__ as g; g.build()"
step pytest_gpu 600 python -m pytest tests -q -m gpu
step bench 300 python bench.py --steps 20 --warmup 5
step bench_bert 300 python bench.py --model bert --steps 20 --warmup 5
step stream 300 python examples/resnet50_stream.py --records 20480 --batch 256
cd /tmp && export TMPDIR=/tmp
step rocprof_bert 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bert" -o run -- python "$REPO/bench.py" --model bert --steps 5 --warmup 2
