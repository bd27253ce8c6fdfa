source tools/gpu_calls/gpu_steps.sh
step pytest_compiler 600 python -u -m pytest tests/test_compiler.py tests/test_arena.py tests/test_fp8.py -x -v -m gpu --timeout 300 --timeout-method thread
step bench_resnet 500 python bench.py --steps 30 --warmup 5
step bench_inc_fp8 500 python bench.py --model inception_v3 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
step rocprof_rn 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rn" -o run -- python "$REPO/bench.py" --steps 5 --warmup 2
step rocprof_inc 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_inc" -o run -- python "$REPO/bench.py" --model inception_v3 --steps 5 --warmup 2
