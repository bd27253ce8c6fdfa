# round 2, session 4: validation after the stem / dconv / preprocess changes
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_resnet_default 300 python -u bench.py
step bench_resnet 300 python -u bench.py --steps 300 --warmup 10
step bench_bert 300 python -u bench.py --model bert --steps 100 --warmup 5
step bench_bert_graph 300 python -u bench.py --model bert_graph --steps 30 --warmup 5
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
step bench_inc 300 python -u bench.py --model inception_v3 --steps 100 --warmup 5
step bench_inc_dyn 300 python -u bench.py --model inception_v3 --steps 50 --warmup 5 --dynamic
step bench_rn_open 300 python -u bench.py --steps 200 --warmup 20 --offered-rate 40000 --buckets 32,64,96,128,160,192,224,256
step rn_stream_sm 300 python -u examples/resnet50_stream.py --records 100000 --savedmodel
step layers 300 python -u bench/layer_table.py --model resnet50
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step prof_resnet 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rn_final" -o rn -- python3 bench.py --steps 10 --warmup 3
