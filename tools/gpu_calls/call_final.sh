# Round validation: GPU tests, smoke, every bench model, ResNet + Inception kernel profiles
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_resnet 500 python bench.py --steps 30 --warmup 5
step bench_resnet_b384 500 python bench.py --steps 30 --warmup 5 --batch 384
step bench_bert 500 python bench.py --model bert --steps 30 --warmup 5
step bench_wd 500 python bench.py --model widedeep --steps 50 --warmup 10
step bench_inc_fp8 500 python bench.py --model inception_v3 --steps 20 --warmup 5
step bench_inc_dyn 500 python bench.py --model inception_v3 --steps 20 --warmup 5 --buckets 64,128 --dynamic
cd /tmp && export TMPDIR=/tmp
step rocprof_rn 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rn" -o run -- python "$REPO/bench.py" --steps 5 --warmup 2
step rocprof_bert 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bert" -o run -- python "$REPO/bench.py" --model bert --steps 5 --warmup 2
