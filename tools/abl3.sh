# Ablation in the default (fused, 3-stream) configuration: which part bounds the step.
# dbg bits: 1 = no k_pred passes, 8|16 = no residual reads in k_pred, 65536 = no LF filtering.
set -e
mkdir -p gpurun_out
for d in ${DBGS:-0 1 65536 65537 24}; do
  VP9HIP_DEBUG=$d timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/abl3_$d.log 2>&1
  echo "dbg=$d $(python -c "import json;d=json.loads(open('gpurun_out/abl3_$d.log').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")"
done
