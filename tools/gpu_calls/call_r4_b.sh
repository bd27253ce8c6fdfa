# round 4 B: the GPU suite again (after the ws=1 W&D capture fix), the per-layer ResNet-50
# table, the other BASELINE models, the coordinator -> 8 workers transport (relocated source
# vs coordinator-produced), and an Inception-v3 fp8 kernel trace analysed per replay
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread
step layers_rn 400 python -u tools/layer_table.py --reps 5 --out "$OUT/layers_rn.md"
step bench_inc 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step bench_inc_dyn 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
step bench_bert_graph 300 python -u bench.py --model bert_graph --steps 30 --warmup 5
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
step transport8 300 python -u bench/transport_bench.py --workers 8 --records 60000
step transport8_coord 300 python -u bench/transport_bench.py --workers 8 --records 30000 --no-relocate
cd /tmp && export TMPDIR=/tmp
step rocprof_inc 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_inc" -o run -- python "$REPO/bench.py" --model inception_v3 --steps 20 --warmup 3
