# operator chaining: BERT / ResNet-50 streams
source tools/gpu_calls/gpu_steps.sh
step bert_stream_pipe 300 python -u examples/bert_stream.py --records 131072 --batch 256
step bert_stream_l3 300 python -u examples/bert_stream.py --records 131072 --batch 256 --lanes 3
step rn_stream_sm 300 python -u examples/resnet50_stream.py --records 100000 --savedmodel
step rn_stream_zoo 300 python -u examples/resnet50_stream.py --records 100000
step rn_stream_proc 300 python -u examples/resnet50_stream.py --records 100000 --processes
