# GPU suite re-run after the torchrun record-parsing fix
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu2 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
step bert_stream 300 python -u examples/bert_stream.py --records 196608 --batch 256 --steady
