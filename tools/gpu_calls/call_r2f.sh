# SignatureBatchedModel: GPU test, BERT / ResNet-50 SavedModel streams on the pipelined runner
source tools/gpu_calls/gpu_steps.sh
step sbm_test 300 python -u -m pytest tests/test_model_function_compiled.py -x -v -m gpu --timeout 200 --timeout-method thread
step bert_stream_pipe 300 python -u examples/bert_stream.py --records 65536 --batch 256
step bert_stream_sync 300 python -u examples/bert_stream.py --records 16384 --batch 256 --sync
step rn_stream_sm 300 python -u examples/resnet50_stream.py --records 60000 --savedmodel
step rn_stream_zoo 300 python -u examples/resnet50_stream.py --records 60000
