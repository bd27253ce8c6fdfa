# round 4 D: the per-layer ResNet-50 table (B=256, and the plan at 32 / 64 images: Infinity-
# Cache residency of stage-1 tensors), the chain's layer table, SQ counters of conv_lite and
# the 8-wave tile on the stage-3 3x3, and call B's
# leftovers (other BASELINE models, coordinator -> 8 workers transport)
source tools/gpu_calls/gpu_steps.sh
step layers_rn 300 python -u tools/layer_table.py --reps 5 --out "$OUT/layers_rn.md"
FT_CHAIN_BATCH=32 step layers_chain32 300 python -u tools/layer_table.py --reps 5 --out "$OUT/layers_chain32.md"
step layers_rn_b32 300 python -u tools/layer_table.py --batch 32 --reps 9 --out "$OUT/layers_rn_b32.md"
step bench_inc_dyn 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
step bench_bert_graph 300 python -u bench.py --model bert_graph --steps 30 --warmup 5
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
step transport8 300 python -u bench/transport_bench.py --workers 8 --records 60000
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
for I in lite lite8s3; do
  step pmc_s3_$I 120 timeout -s KILL 60 rocprofv3 --pmc $SQ --output-format csv -d "$OUT/pmc_s3_$I" -o run -- python "$REPO/bench/conv_layer_probe.py" --layers s3_3x3 --impls $I --reps 5
done
