# round 4 A: the driver's GPU suite (start barrier + isolated multi-subtask test), smoke
# (now checked against the fp32 interpreter), the headline bench, the 3x3 conv tile
# variants per layer and in the bench, a ResNet-50 kernel profile
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step probe_layers 300 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3,s3_3x3s2 --impls lite,lite256,lite256s3,lites3 --reps 20
step bench_rn_a 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_rn_auto 300 env FT_CONV_LITE_TILE=auto python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_rn_t5 300 env FT_CONV_LITE_TILE=5 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_rn_b 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_rn_auto300 300 env FT_CONV_LITE_TILE=auto python -u bench.py --gpus 1 --steps 300 --warmup 10
step bench_rn_300 300 python -u bench.py --gpus 1 --steps 300 --warmup 10
cd /tmp && export TMPDIR=/tmp
step rocprof_rn 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rn" -o run -- python "$REPO/bench.py" --steps 5 --warmup 2
