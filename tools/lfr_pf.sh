# k_lfr next-SB interior prefetch (VP9HIP_LFR_PF) on/off on the inter configs (GPU box).
set -e
mkdir -p gpurun_out
for pf in 0 1; do for c in C2 C5; do
  VP9HIP_LFR_PF=$pf timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pf${pf}_$c.json 2> gpurun_out/pf${pf}_$c.err
  echo "pf=$pf $c $(python -c "import json;d=json.loads(open('gpurun_out/pf${pf}_$c.json').read().strip().split(chr(10))[-1]);print(d['value'], d['roofline']['kernel_ms']['k_lfr'])")"
done; done
