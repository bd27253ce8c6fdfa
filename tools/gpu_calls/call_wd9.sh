# W&D: one shared sort for both tables, fused mask+bias-grad
source tools/gpu_calls/gpu_steps.sh
step wd_tests 400 python -u -m pytest tests/test_widedeep.py tests/test_rccl.py -x -q -m gpu --timeout 350 --timeout-method thread
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
step bench_wd_b 300 python -u bench.py --model widedeep --steps 50 --warmup 10
cd /tmp && export TMPDIR=/tmp
step prof_wd 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_wd7" -o run -- python "$REPO/bench.py" --model widedeep --steps 20 --warmup 5
