#!/bin/bash
# round 5 V: the lane-phase test and the arena / engine GPU tests; the headline bench with
# the new default lane offset.
OUT=gpurun_out/r05_v
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
step tests 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_arena.py
step bench 150 python bench.py
step bench2 150 python bench.py
echo done >&2
