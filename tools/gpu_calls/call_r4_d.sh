# round 4 D: the per-layer ResNet-50 table (B=256) and the batch-slice chain's table
# (32-image slices: per-step time summed over the slices); SQ counters of conv_lite on the
# stage-3 3x3; Inception-v3 fp8 with conv_lite_fp8's eight-wave three-stage tile (cfg 9)
# and with the stem chained; call B's leftovers (other BASELINE models, 8-worker transport)
source tools/gpu_calls/gpu_steps.sh
step layers_rn 300 python -u tools/layer_table.py --reps 5 --out "$OUT/layers_rn.md"
FT_CHAIN_BATCH=32 step layers_chain32 300 python -u tools/layer_table.py --reps 5 --out "$OUT/layers_chain32.md"
step test_fp8 300 python -u -m pytest tests/test_fp8.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
if grep -q " passed" "$OUT/test_fp8.log" && ! grep -q "failed" "$OUT/test_fp8.log"; then
  step layers_inc 300 python -u tools/layer_table.py --model inception_v3 --reps 5 --out "$OUT/layers_inc.md"
  FT_FP8_LITE_WIDE=256 step layers_inc_wide 300 python -u tools/layer_table.py --model inception_v3 --reps 5 --out "$OUT/layers_inc_wide.md"
  step bench_inc 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
  FT_FP8_LITE_WIDE=256 step bench_inc_wide256 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
  FT_CHAIN_BATCH=32 FT_CHAIN_MIN_HW=5041 FT_CHAIN_EDGE=1 step bench_inc_chain32 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
fi
step bench_inc_dyn 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
step bench_bert_graph 300 python -u bench.py --model bert_graph --steps 30 --warmup 5
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
step transport8 300 python -u bench/transport_bench.py --workers 8 --records 60000
cd /tmp && export TMPDIR=/tmp
step pmc_list 60 timeout -s KILL 50 rocprofv3 -L
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
step pmc_s3_lite 120 timeout -s KILL 60 rocprofv3 --pmc $SQ --output-format csv -d "$OUT/pmc_s3_lite" -o run -- python "$REPO/bench/conv_layer_probe.py" --layers s3_3x3 --impls lite --reps 5
