# ResNet-50 stream: micro-batch sweep (L3 residency of inter-layer activations vs launch fill)
source tools/gpu_calls/gpu_steps.sh
for b in 64 128 192 256 384 512; do
  step bench_b$b 300 python bench.py --steps 30 --warmup 5 --batch $b
done
