# W&D on gemm_train: tests, bench, kernel profile; gemm_train kernel-level stats
source tools/gpu_calls/gpu_steps.sh
step pytest_wd 300 python -u -m pytest tests/test_widedeep.py -q -x --timeout 120 --timeout-method thread -m gpu
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step prof_wd 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_wd" -o wd -- python3 bench.py --model widedeep --steps 20 --warmup 5
step prof_gt 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_gt" -o gt -- python3 bench/gemm_train_bench.py
