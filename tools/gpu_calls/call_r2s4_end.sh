# round 2 session 4, end: GPU suite, smoke, headline + secondary benches on the final tree
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_resnet_default 300 python -u bench.py
step bench_resnet 300 python -u bench.py --steps 300 --warmup 10
step bench_inc 300 python -u bench.py --model inception_v3 --steps 100 --warmup 5
step bench_bert 300 python -u bench.py --model bert --steps 100 --warmup 5
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step prof_resnet 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rn_end" -o rn -- python3 bench.py --steps 10 --warmup 3
