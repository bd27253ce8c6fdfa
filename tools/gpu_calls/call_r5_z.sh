#!/bin/bash
# round 5 Z: job mode with the lane offset (tests + bench --job twice), headline once.
OUT=gpurun_out/r05_z
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
step tests 400 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_job_dp.py tests/test_examples.py
step job 200 python bench.py --job
step job_o0 200 python bench.py --job --lane-offset-us 0
step job2 200 python bench.py --job
step rn 150 python bench.py
echo done >&2
