# round 3 (session 3) I: batches in flight = lanes + 1 (depth 3 at two lanes) instead of the
# old floor lanes + 2: p50 latency vs throughput in the driver's window and at 300 steps
source tools/gpu_calls/gpu_steps.sh
for i in a b; do
  step d3_$i 300 python -u bench.py --steps 20 --warmup 5
  step d4_$i 300 python -u bench.py --steps 20 --warmup 5 --depth 4
done
step d3_300 300 python -u bench.py --steps 300 --warmup 10
step d4_300 300 python -u bench.py --steps 300 --warmup 10 --depth 4
step inc_d3 300 python -u bench.py --model inception_v3 --steps 100 --warmup 10
step inc_d4 300 python -u bench.py --model inception_v3 --steps 100 --warmup 10 --depth 4
step bert_d4 300 python -u bench.py --model bert_graph --steps 50 --warmup 5
step bert_d5 300 python -u bench.py --model bert_graph --steps 50 --warmup 5 --depth 5
