source tools/gpu_calls/gpu_steps.sh
step pytest_remote 300 python -u -m pytest tests/test_remote.py -x -v -m gpu --timeout 200 --timeout-method thread
step tune_bert 600 python -u bench/tune_bert_gemms.py --out gpurun_out/tunableop_gfx950.csv
step tune_cmp 300 python -u bench/tune_bert_gemms.py --out gpurun_out/tunableop_gfx950.csv --compare
