# round 4 C: conv_lite tile variants after the raw-s_barrier fix of the 3-stage loop (the
# __syncthreads of the first try drained the third stage): 4-wave 128x128 / 256x128 with
# 3 stages, and the new 8-wave 256x128 tile (2 waves per SIMD) with 3 / 2 stages, vs the
# default per layer; SQ counters of the default and the 8-wave tile on the stage-3 3x3;
# then the plan at micro-batch 32 / 64 (Infinity-Cache residency of stage-1 tensors)
source tools/gpu_calls/gpu_steps.sh
step test_conv 300 python -u -m pytest tests/test_conv_pp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
if ! grep -q " passed" "$OUT/test_conv.log" || grep -q "failed" "$OUT/test_conv.log"; then
  echo "[call] conv tests did not pass; no probes"; exit 1
fi
step probe_3x3 300 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3,s3_3x3s2 --impls lite,lites3,lite256s3,lite8s3,lite8 --reps 20
step probe_1x1 300 python -u bench/conv_layer_probe.py --layers s2_reduce,s3_reduce,s4_expand,s1_reduce --impls igemm,lite,lite8s3,lite8 --reps 20
step test_chain 300 python -u -m pytest tests/test_chain.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
if grep -q " passed" "$OUT/test_chain.log" && ! grep -q "failed" "$OUT/test_chain.log"; then
  step bench_default 300 python -u bench.py --steps 20 --warmup 5
  FT_CHAIN_BATCH=32 step bench_chain32 300 python -u bench.py --steps 20 --warmup 5
  FT_CHAIN_BATCH=64 step bench_chain64 300 python -u bench.py --steps 20 --warmup 5
  FT_CHAIN_BATCH=16 step bench_chain16 300 python -u bench.py --steps 20 --warmup 5
  FT_CONV_LITE_EXPAND=1 step bench_lite_expand 300 python -u bench.py --steps 20 --warmup 5
  FT_CHAIN_BATCH=32 FT_CHAIN_EDGE=1 step bench_chain32e 300 python -u bench.py --steps 20 --warmup 5
  step bench_inc 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
  FT_CHAIN_BATCH=32 FT_CHAIN_MIN_HW=5041 FT_CHAIN_EDGE=1 step bench_inc_chain32 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
  FT_CHAIN_BATCH=32 step layers_chain32 300 python -u tools/layer_table.py --reps 5 --out "$OUT/layers_chain32.md"
fi
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
for I in lite lite8s3; do
  step pmc_s3_$I 120 timeout -s KILL 60 rocprofv3 --pmc $SQ --output-format csv -d "$OUT/pmc_s3_$I" -o run -- python "$REPO/bench/conv_layer_probe.py" --layers s3_3x3 --impls $I --reps 5
done
cd "$REPO"
# Infinity-Cache residency probe: the same plan at micro-batch 32 (each step's inputs were
# written one or two steps earlier: ~13-51 MB per stage-1 tensor, resident in the 256 MiB L3)
# against 256 (411 MB per stage-1 tensor: every read goes to HBM); x8 per-step sums compare
step layers_rn_b32 300 python -u tools/layer_table.py --batch 32 --reps 9 --out "$OUT/layers_rn_b32.md"
step layers_rn_b64 300 python -u tools/layer_table.py --batch 64 --reps 9 --out "$OUT/layers_rn_b64.md"
