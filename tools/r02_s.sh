# batches in flight 1 vs 2 on C3 / C2 / C5 with k_lfrd + wave-per-unit MC
set -e
mkdir -p gpurun_out
line() { python -c "import json;d=json.loads(open('$1').read().strip().split(chr(10))[-1]);print('$2', d['value'], d['ms_per_step'], d.get('verified_frames'))"; }
for c in C3 C2 C5; do
  for i in 1 2; do
    timeout -k 10 300 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline --inflight $i > gpurun_out/r02s_${c}_$i.json 2> gpurun_out/r02s_${c}_$i.err
    line gpurun_out/r02s_${c}_$i.json ${c}_inflight$i
  done
done
