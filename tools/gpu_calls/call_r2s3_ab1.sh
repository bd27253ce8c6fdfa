# A/B: row-band preprocess kernel + decimated stage-1 -> stage-2 tail output vs the previous kernels
source tools/gpu_calls/gpu_steps.sh
step pytest_sel 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_bottleneck.py tests/test_kernels_gpu.py tests/test_compiler.py tests/test_fullsize_numerics.py
step ab_old1 300 env FTM_TAIL_DECIMATE=0 FTM_PRE_ROWS=0 python -u bench.py --steps 40 --warmup 5
step ab_new1 300 python -u bench.py --steps 40 --warmup 5
step ab_old2 300 env FTM_TAIL_DECIMATE=0 FTM_PRE_ROWS=0 python -u bench.py --steps 40 --warmup 5
step ab_new2 300 python -u bench.py --steps 40 --warmup 5
step ab_pre_old 300 env FTM_PRE_ROWS=0 python -u bench.py --steps 40 --warmup 5
step inc_new 300 python -u bench.py --model inception_v3 --steps 20 --warmup 5
step inc_old 300 env FTM_PRE_ROWS=0 python -u bench.py --model inception_v3 --steps 20 --warmup 5
step layers 300 python -u bench/layer_table.py --model resnet50
cd /tmp && export TMPDIR=/tmp
step prof_rn 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rn" -o rn -- python3 -u "$REPO/bench.py" --steps 10 --warmup 3
