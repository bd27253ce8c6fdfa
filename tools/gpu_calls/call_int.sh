# gemm_pp integration: GPU tests of the touched models, both benches, kernel stats
source tools/gpu_calls/gpu_steps.sh
step pytest_int 600 python -u -m pytest tests/test_gemm_pp.py tests/test_bert.py tests/test_compiler.py tests/test_bottleneck.py -x -q -m gpu --timeout 120 --timeout-method thread
step bench_rn 300 python -u bench.py --steps 30 --warmup 5
step bench_bert 300 python -u bench.py --model bert --steps 30 --warmup 5
cd /tmp && export TMPDIR=/tmp
step prof_bert 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_bert -o run -- python3 $REPO/bench.py --model bert --steps 10 --warmup 3
step prof_rn 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_rn -o run -- python3 $REPO/bench.py --steps 10 --warmup 3 --lanes 1
