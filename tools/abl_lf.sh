set -e
mkdir -p gpurun_out
for d in 0 1 3 7; do
  VP9HIP_STREAMS=1 VP9HIP_DEBUG=$(( d << 16 )) timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/alf_$d.log 2>&1
  echo "lfdbg=$d $(python -c "import json;d=json.loads(open('gpurun_out/alf_$d.log').read().strip().split(chr(10))[-1]);print(d['roofline']['kernel_ms'])")"
done
