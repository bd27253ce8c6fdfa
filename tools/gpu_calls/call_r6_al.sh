#!/bin/bash
# Round 6 call AL: LDS counters of the stage-3 3x3 conv_lite (VERDICT r5 #1 asked for them).
source tools/gpu_calls/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp
step r06_al/pmc_lds 90 timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY -d "$OUT/r06_al/pmc_lds" -o run --output-format csv -- python "$REPO/bench/conv_layer_probe.py" --layers s3_3x3 --impls lite:2 --reps 5
