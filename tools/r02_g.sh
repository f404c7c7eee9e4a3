# C3 with 1 / 2 batches in flight
set -e
mkdir -p gpurun_out
line() { python -c "import json;d=json.loads(open('$1').read().strip().split(chr(10))[-1]);print('$2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --inflight $i > gpurun_out/r02g_C3_$i.json 2> gpurun_out/r02g_C3_$i.err
  line gpurun_out/r02g_C3_$i.json C3_inflight$i
done
