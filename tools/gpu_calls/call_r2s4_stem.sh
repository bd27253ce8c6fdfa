# 8-wave pooled stem tiles (14 x 8 pooled pixels per workgroup) vs the 4-wave 7 x 8 tiles
source tools/gpu_calls/gpu_steps.sh
step pytest_dconv 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_dconv.py
step stem_ab 120 python -u bench/stem_ab.py
step ab7_1 300 env FTM_STEM_POOL_ROWS=7 python -u bench.py --steps 40 --warmup 5
step ab14_1 300 env FTM_STEM_POOL_ROWS=14 python -u bench.py --steps 40 --warmup 5
step ab7_2 300 env FTM_STEM_POOL_ROWS=7 python -u bench.py --steps 40 --warmup 5
step ab14_2 300 env FTM_STEM_POOL_ROWS=14 python -u bench.py --steps 40 --warmup 5
