# round 3 (session 2) A: GPU suite on the restored tree + packed BERT test, smoke, default bench, ResNet kernel trace
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 780 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_resnet_default 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step prof_rn 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rn" -o rn -- python3 bench.py --gpus 1 --steps 20 --warmup 5
