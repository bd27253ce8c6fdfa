#!/bin/bash
# round 5 P: ResNet-50 — the stage-4 identity-residual expands (512 -> 2048) on gemm_pp with its
# residual epilogue, and the stage-2 reduces (512 -> 128) on gemm_pp; interleaved.
OUT=gpurun_out/r05_p
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
for r in 1 2; do
  step base_$r 150 python bench.py
  step ppres_$r 150 env FTM_AB_PP_RES=1 python bench.py
  step ppn128_$r 150 env FTM_AB_PP_N128=1 python bench.py
  step both_$r 150 env FTM_AB_PP_RES=1 FTM_AB_PP_N128=1 python bench.py
done
step layers_both 300 env FTM_AB_PP_RES=1 FTM_AB_PP_N128=1 python -u tools/layer_table.py --model resnet50 --reps 3 --out "$OUT/layers_both.md"
step smoke_both 150 env FTM_AB_PP_RES=1 FTM_AB_PP_N128=1 python -c "import __graft_entry__ as g; g.smoke()"
echo done >&2
