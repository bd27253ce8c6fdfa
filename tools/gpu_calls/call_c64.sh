source tools/gpu_calls/gpu_steps.sh
step pytest_c64 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu -k conv3x3_c64 --timeout 120 --timeout-method thread
step pytest_comp 300 python -u -m pytest tests/test_compiler.py tests/test_arena.py -x -v -m gpu --timeout 200 --timeout-method thread
step bench_resnet 300 python bench.py --steps 30 --warmup 5
step bench_resnet_off 300 env FTM_CONV3X3C64=0 python bench.py --steps 30 --warmup 5
cd /tmp && export TMPDIR=/tmp
step rocprof_rn 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rn" -o run -- python "$REPO/bench.py" --steps 5 --warmup 2
