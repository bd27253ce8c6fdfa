# GPU tests incl. worker-process ResNet subtasks + BERT profile for the packing work
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread
cd /tmp && export TMPDIR=/tmp
step rocprof_bert 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bert" -o run -- python "$REPO/bench.py" --model bert --steps 5 --warmup 2
