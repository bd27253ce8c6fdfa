# round 2, session 4 re-entry: rebuilt tree validation (GPU suite, smoke, headline bench, kernel stats)
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_resnet 300 python -u bench.py --steps 40 --warmup 5
step bench_bert 300 python -u bench.py --model bert --steps 30 --warmup 5
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step prof_resnet 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rn" -o rn -- python3 bench.py --steps 10 --warmup 3
