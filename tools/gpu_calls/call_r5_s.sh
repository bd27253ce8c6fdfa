#!/bin/bash
# round 5 S: the headline's 20-step window batch by batch (bench.py --timeline), three runs.
OUT=gpurun_out/r05_s
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
for r in 1 2 3; do
  step win_$r 150 python bench.py --timeline
done
step win_300 200 python bench.py --timeline --steps 300
echo done >&2
