# round 3 (session 3) A: re-validate the restored tree: GPU suite, smoke, the driver's
# default bench (x2), ResNet-50 kernel stats, Inception-v3 fp8 / BERT graph / W&D benches
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_rn_a 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_rn_b 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step prof_rn 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rn" -o rn -- python3 bench.py --gpus 1 --steps 20 --warmup 5
step bench_inc 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step bench_bert_graph 400 python -u bench.py --model bert_graph --steps 50 --warmup 5
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
