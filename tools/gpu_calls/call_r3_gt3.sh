# W&D: radix sort without hot-key atomics, parallel colsum, 4-stage gemm_train for small grids
source tools/gpu_calls/gpu_steps.sh
step pytest_gt 300 python -u -m pytest tests/test_gemm_train.py tests/test_widedeep.py -q -x --timeout 120 --timeout-method thread -m gpu
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step prof_wd 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_wd3" -o wd -- python3 bench.py --model widedeep --steps 20 --warmup 5
step bench_rn_a 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_rn_b 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_rn_300 300 python -u bench.py --gpus 1 --steps 300 --warmup 10
