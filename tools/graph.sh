set -e
mkdir -p gpurun_out
for g in 0 1; do
  VP9HIP_GRAPH=$g timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/gr_$g.log 2>&1
  echo "graph=$g $(python -c "import json;d=json.loads(open('gpurun_out/gr_$g.log').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")"
done
