# full-size numerics, slab transport diagnostics
source tools/gpu_calls/gpu_steps.sh
step pytest_num 600 python -u -m pytest tests/test_fullsize_numerics.py -x -v -s -m gpu --timeout 300 --timeout-method thread
FTM_SLAB_DEBUG=1 step transport_slab 300 python -u bench/transport_bench.py --workers 8 --records 200000
FTM_SLAB_BYTES=0 step transport_pickle 300 python -u bench/transport_bench.py --workers 8 --records 200000
FTM_SLAB_DEBUG=1 step transport_slab4 300 python -u bench/transport_bench.py --workers 4 --records 200000
FTM_SLAB_BYTES=0 step transport_pickle4 300 python -u bench/transport_bench.py --workers 4 --records 200000
