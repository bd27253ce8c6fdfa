#!/bin/bash
# round 5 D: new kernels first (pool+1x1 fp8, bucketed exchange capture, lockstep fused
# step, bench --job P=1), then the whole GPU suite, smoke, and the benches (ResNet-50 SPMD
# and job mode, Inception-v3 fp8 static).  Every GPU step has its own time limit; a crash,
# abort or time-out ends the call (no later GPU step runs).
OUT=gpurun_out/r05_d
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
step new_tests 400 $PYT -m gpu tests/test_fp8.py::test_pool_conv1x1_fp8_gpu tests/test_fp8.py::test_inception_v3_fp8_plan_gpu tests/test_rccl.py tests/test_lockstep.py tests/test_job_dp.py
step gpu_suite 780 $PYT -m gpu tests --maxfail 10
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_rn 150 python bench.py
step bench_job 200 python bench.py --job
step bench_inc 200 python bench.py --model inception_v3 --steps 30 --warmup 5
export TMPDIR=/tmp
R=$(pwd)
step layers_inc 300 python -u tools/layer_table.py --model inception_v3 --reps 3 --out "$OUT/layers_inc.md"
step wd_trace 300 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats -d $R/$OUT/wd_prof -o wd -- python3 $R/tools/wd_bucketed_trace.py"
echo done >&2
