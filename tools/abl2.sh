# k_pred / k_lf ablation with separate launches on one stream (VP9HIP_PLF=0, 1 group)
set -e
mkdir -p gpurun_out
for d in 0 8 16 24 1 65536 131072; do
  VP9HIP_PLF=0 VP9HIP_STREAMS=1 VP9HIP_DEBUG=$d timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abl_$d.log 2>&1
  echo "dbg=$d $(python -c "import json;d=json.loads(open('gpurun_out/abl_$d.log').read().strip().split(chr(10))[-1]);print(d['value'], d['roofline']['kernel_ms'])")"
done
