#!/bin/bash
# round 5 E: pool+1x1 fp8 kernel v2 (numerics + A/B microbench), the fixes of call D's
# failures (fused agreed step with partial pieces, multi-output fp8 test, smoke), the
# interleaved head launches (test + bench A/B), then the GPU suite.
OUT=gpurun_out/r05_e
mkdir -p "$OUT"
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "[step] $name" >&2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> "$OUT/rc.txt"
  if [ $rc -gt 1 ]; then echo "[step] $name ended with $rc: stopping" >&2; exit $rc; fi
  return 0
}
PYT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
step fixes 400 $PYT -m gpu tests/test_fp8.py::test_pool_conv1x1_fp8_gpu tests/test_fp8.py::test_conv_fp8_multi_output_gpu tests/test_lockstep.py tests/test_widedeep.py::test_fused_step_partial_batch_gpu tests/test_arena.py::test_interleaved_head_pieces_match_whole_batch_gpu tests/test_rccl.py
step poolconv_bench 120 python -u bench/pool_conv_bench.py
step poolconv_bench32 120 python -u bench/pool_conv_bench.py --batch 32
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step rn_inter 150 python bench.py
step rn_nointer 150 python bench.py --no-interleave
step rn_inter2 150 python bench.py
step rn_nointer2 150 python bench.py --no-interleave
step inc 200 python bench.py --model inception_v3 --steps 30 --warmup 5
step inc_nopc 200 env FT_POOL_CONV_FUSION=0 python bench.py --model inception_v3 --steps 30 --warmup 5
step wd_trace 200 python -u tools/wd_bucketed_trace.py
step wd_bench 200 python bench.py --model widedeep
step gpu_suite 780 $PYT -m gpu tests --maxfail 10
echo done >&2
