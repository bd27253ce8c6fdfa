# Preprocess head on the H2D staging slot (no D2D input copy): GPU tests, benches, kernel trace
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step bench_resnet_a 300 python bench.py --steps 40 --warmup 8
step bench_resnet_b 300 python bench.py --steps 40 --warmup 8
step bench_inc_fp8 300 python bench.py --model inception_v3 --steps 30 --warmup 5
cd /tmp && export TMPDIR=/tmp
step rocprof_rn 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_head" -o run -- python "$REPO/bench.py" --steps 5 --warmup 2
