# round 3 (session 2) O: worker-process model operator chained as the tail of the source's
# chain (--processes), transport with chaining, and Inception-v3 fp8 dynamic batching with
# finer buckets (padding to the bucket is the main dynamic-vs-static loss)
source tools/gpu_calls/gpu_steps.sh
step stream_proc 300 python -u examples/resnet50_stream.py --records 200000 --processes
step transport8 300 python -u bench/transport_bench.py --workers 8 --records 80000
step inc_static 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_dyn32 300 python -u bench.py --model inception_v3 --steps 60 --warmup 10 --dynamic
step inc_dyn16 400 python -u bench.py --model inception_v3 --steps 60 --warmup 10 --dynamic --buckets 64,80,96,112,128,144,160,176,192,208,224,240
step inc_dyn8 500 python -u bench.py --model inception_v3 --steps 60 --warmup 10 --dynamic --buckets 64,72,80,88,96,104,112,120,128,136,144,152,160,168,176,184,192,200,208,216,224,232,240,248
