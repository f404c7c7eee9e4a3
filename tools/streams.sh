# Frame-group streams sweep on C3 (VP9HIP_STREAMS).
set -e
mkdir -p gpurun_out
for s in ${SWEEP:-1 2 3 4}; do
  VP9HIP_STREAMS=$s timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > gpurun_out/st_$s.json 2> gpurun_out/st_$s.err
  echo "streams=$s $(python -c "import json;d=json.loads(open('gpurun_out/st_$s.json').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'])")"
done
