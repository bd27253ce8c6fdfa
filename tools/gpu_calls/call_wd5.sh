# fused Wide&Deep step v2 (slice segment sum, parallel loss, library dX + mask)
source tools/gpu_calls/gpu_steps.sh
step wd_tests 300 python -u -m pytest tests/test_widedeep.py tests/test_gemm_pp.py -x -q -m gpu --timeout 200 --timeout-method thread
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
step bench_wd_b 300 python -u bench.py --model widedeep --steps 50 --warmup 10
cd /tmp && export TMPDIR=/tmp
step prof_wd 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_wd4" -o run -- python "$REPO/bench.py" --model widedeep --steps 20 --warmup 5
