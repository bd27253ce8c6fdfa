source tools/gpu_calls/gpu_steps.sh
step pytest_dual 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_bottleneck.py tests/test_compiler.py tests/test_arena.py -x -v -m gpu -k "bottleneck or plan or arena or lanes" --timeout 200 --timeout-method thread
step bench_rn 300 python bench.py --steps 30 --warmup 5
step bench_rn_nofuse 300 env FTM_TAIL_FUSE=0 python bench.py --steps 30 --warmup 5
step bench_rn2 300 python bench.py --steps 30 --warmup 5
cd /tmp && export TMPDIR=/tmp
step rocprof_rn 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rn_dual" -o run -- python "$REPO/bench.py" --steps 5 --warmup 2 --lanes 1
