#!/bin/bash
# round 5 final, part 2: the headline (driver window and 300 steps), the job mode, Inception
# fp8 static / dynamic, per-layer tables, and the headline's kernel stats under rocprofv3.
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$REPO/gpurun_out/r05_final2"
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
step bench_rn 150 python bench.py
step bench_rn2 150 python bench.py
step bench_rn_300 200 python bench.py --steps 300
step bench_job 200 python bench.py --job
step bench_inc 200 python bench.py --model inception_v3 --steps 30 --warmup 5
step bench_inc2 200 python bench.py --model inception_v3 --steps 30 --warmup 5
step bench_inc_dyn 200 python bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
step bench_inc_l2 200 python bench.py --model inception_v3 --steps 30 --warmup 5 --lanes 2
step bench_wd 200 python bench.py --model widedeep --steps 50 --warmup 10
step layers_rn 300 python -u tools/layer_table.py --model resnet50 --reps 3 --out "$OUT/layers_rn.md"
step layers_inc 300 python -u tools/layer_table.py --model inception_v3 --reps 3 --out "$OUT/layers_inc.md"
cd /tmp && export TMPDIR=/tmp
step prof_rn 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rn" -o run -- python "$REPO/bench.py" --steps 20 --warmup 5
echo done >&2
