#!/bin/bash
# round 5 X: the final ResNet-50 plan's fabric bytes per batch (FETCH_SIZE / WRITE_SIZE, one
# lane, separate passes) and MFMA busy share, for the round-5 profile record.
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$REPO/gpurun_out/r05_x"
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
cd /tmp && export TMPDIR=/tmp
step pmc_fetch 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 "$REPO/bench.py" --gpus 1 --steps 3 --warmup 1 --lanes 1
step pmc_write 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- python3 "$REPO/bench.py" --gpus 1 --steps 3 --warmup 1 --lanes 1
step pmc_sq 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_sq" -o run -- python3 "$REPO/bench.py" --gpus 1 --steps 3 --warmup 1 --lanes 1
cd "$REPO" && python3 tools/tcc_bytes.py "$OUT/pmc_fetch" "$OUT/pmc_write" > "$OUT/tcc_bytes.txt" 2>&1
echo done >&2
