# round 3 start: GPU suite on the tree with the bench self-launch + ADVICE fixes, default bench
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread
step bench_resnet_default 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
step launch_check 120 python -u bench.py --gpus 2 --rehearse-fake-comm --launch-check
