source tools/gpu_calls/gpu_steps.sh
step pytest_pre 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8.py tests/test_compiler.py -x -v -m gpu -k "preprocess or inception or plan" --timeout 200 --timeout-method thread
step bench_inc 300 python bench.py --model inception_v3 --steps 30 --warmup 5
step bench_rn 300 python bench.py --steps 30 --warmup 5
cd /tmp && export TMPDIR=/tmp
step rocprof_inc 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_inc_pre" -o run -- python "$REPO/bench.py" --model inception_v3 --steps 5 --warmup 2 --lanes 1
step rocprof_rn 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rn_pre" -o run -- python "$REPO/bench.py" --steps 5 --warmup 2 --lanes 1
