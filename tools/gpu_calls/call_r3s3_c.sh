# round 3 (session 3) C: gather threads per rank (host staging of the micro-batch) in the
# driver's 20-step window: 8 (default) vs 12 vs 16, interleaved
source tools/gpu_calls/gpu_steps.sh
for i in a b c; do
  step g8_$i 300 python -u bench.py --steps 20 --warmup 5
  step g16_$i 300 python -u bench.py --steps 20 --warmup 5 --gather-threads 16
  step g12_$i 300 python -u bench.py --steps 20 --warmup 5 --gather-threads 12
done
step g8_300 300 python -u bench.py --steps 300 --warmup 10
step g16_300 300 python -u bench.py --steps 300 --warmup 10 --gather-threads 16
