# round 4 A: the driver's GPU suite (start barrier + isolated multi-subtask test), smoke
# (now checked against the fp32 interpreter), the headline bench, a ResNet-50 kernel
# profile and the per-layer conv table
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_rn_a 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_rn_b 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step probe_layers 300 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3 --impls lite,pp --reps 20
cd /tmp && export TMPDIR=/tmp
step rocprof_rn 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rn" -o run -- python "$REPO/bench.py" --steps 5 --warmup 2
