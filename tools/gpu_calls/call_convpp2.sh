# conv_pp integrated with measured per-layer selection: tests, A/B bench, kernel stats
source tools/gpu_calls/gpu_steps.sh
step pytest_c 600 python -u -m pytest tests/test_conv_pp.py tests/test_compiler.py tests/test_bottleneck.py tests/test_model_function_compiled.py tests/test_fp8.py -x -q -m gpu --timeout 120 --timeout-method thread
step bench_pp 300 python -u bench.py --steps 30 --warmup 5
FTM_CONV_IMPL=incumbent step bench_inc 300 python -u bench.py --steps 30 --warmup 5
step bench_pp2 300 python -u bench.py --steps 30 --warmup 5
cd /tmp && export TMPDIR=/tmp
step prof_rn 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_rn -o run -- python3 $REPO/bench.py --steps 10 --warmup 3 --lanes 1
