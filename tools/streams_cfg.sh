# Streams sweep on one config (CFG, default C2).
set -e
mkdir -p gpurun_out
for s in ${SWEEP:-2 3 4}; do
  VP9HIP_STREAMS=$s timeout -k 10 300 python bench.py --config ${CFG:-C2} --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sc_$s.json 2> gpurun_out/sc_$s.err
  echo "${CFG:-C2} streams=$s $(python -c "import json;d=json.loads(open('gpurun_out/sc_$s.json').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'])")"
done
