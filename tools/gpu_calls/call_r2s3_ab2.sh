# tail decimation: kernel microbench, GPU tests, end-to-end A/B
source tools/gpu_calls/gpu_steps.sh
step tail_ab 120 python -u bench/tail_decimate_ab.py
step pytest_bn 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_bottleneck.py
step ab_old1 300 env FTM_TAIL_DECIMATE=0 python -u bench.py --steps 40 --warmup 5
step ab_new1 300 python -u bench.py --steps 40 --warmup 5
step ab_old2 300 env FTM_TAIL_DECIMATE=0 python -u bench.py --steps 40 --warmup 5
step ab_new2 300 python -u bench.py --steps 40 --warmup 5
