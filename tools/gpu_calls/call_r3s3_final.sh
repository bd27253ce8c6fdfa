# round 3 (session 3) final (re-run after the gc.freeze change): the committed tree — GPU suite, smoke, the driver's bench (x2),
# ResNet-50 kernel stats, Inception-v3 fp8 / BERT graph / W&D benches, ResNet stream job
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_rn_a 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_rn_b 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_rn_300 300 python -u bench.py --gpus 1 --steps 300 --warmup 10
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step prof_rn 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rn" -o rn -- python3 bench.py --gpus 1 --steps 20 --warmup 5
step bench_inc 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step bench_inc_dyn 500 python -u bench.py --model inception_v3 --steps 60 --warmup 10 --dynamic
step bench_bert_graph 400 python -u bench.py --model bert_graph --steps 50 --warmup 5
step bench_bert 400 python -u bench.py --model bert --steps 50 --warmup 5
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
step stream_rn 400 python -u examples/resnet50_stream.py --records 200000
step launch_check 120 python -u bench.py --gpus 2 --rehearse-fake-comm --launch-check
