# per-layer TFLOP/s and TB/s tables of the compiled ResNet-50 (bf16) and Inception-v3 (fp8) plans
source tools/gpu_calls/gpu_steps.sh
step layers_rn 300 python -u bench/layer_table.py --model resnet50 --jsonl gpurun_out/layers_rn.jsonl
step layers_inc 400 python -u bench/layer_table.py --model inception_v3 --jsonl gpurun_out/layers_inc.jsonl
