source tools/gpu_calls/gpu_steps.sh
step pytest_tail 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_bottleneck.py -x -v -m gpu -k "bottleneck" --timeout 120 --timeout-method thread
step bench_resnet 300 python bench.py --steps 30 --warmup 5
step bench_resnet_off 300 env FTM_TAIL_FUSE=0 python bench.py --steps 30 --warmup 5
cd /tmp && export TMPDIR=/tmp
step rocprof_rn 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_tail" -o run -- python "$REPO/bench.py" --steps 5 --warmup 2 --lanes 1
