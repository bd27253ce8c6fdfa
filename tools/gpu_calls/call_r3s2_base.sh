# round 3 (session 2): GPU suite on the restored tree (gemm_train, LDS radix sort, knob
# cleanup, pinned bundle staging), default bench, W&D bench, kernel stats of both
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_resnet_default 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
step launch_check 120 python -u bench.py --gpus 2 --rehearse-fake-comm --launch-check
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step prof_wd 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_wd" -o wd -- python3 bench.py --model widedeep --steps 20 --warmup 5
step prof_rn 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rn" -o rn -- python3 bench.py --gpus 1 --steps 20 --warmup 5
step bench_bert_graph 400 python -u bench.py --model bert_graph --steps 50 --warmup 5
step bert_stream 400 python -u examples/bert_stream.py --steady --records 16384
