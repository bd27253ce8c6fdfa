#!/bin/bash
# round 5 AA: ResNet-50's remaining generic 1x1 convs (stage-2 reduces, stage-4 expands,
# block1/unit1/conv1) on conv_lite instead of the register-staged igemm; numerics + A/B.
OUT=gpurun_out/r05_aa
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
step smoke_pw 150 env FTM_AB_LITE_PW=1 python -c "import __graft_entry__ as g; g.smoke()"
for r in 1 2 3; do
  step base_$r 150 python bench.py
  step pw_$r 150 env FTM_AB_LITE_PW=1 python bench.py
done
step layers_pw 300 env FTM_AB_LITE_PW=1 python -u tools/layer_table.py --model resnet50 --reps 3 --out "$OUT/layers_pw.md"
echo done >&2
