set -e
mkdir -p gpurun_out
for g in ${GS:-1 2 4}; do
  VP9HIP_STREAMS=$g timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/str_$g.log 2>&1
  echo "streams=$g $(python -c "import json;d=json.loads(open('gpurun_out/str_$g.log').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")"
done
