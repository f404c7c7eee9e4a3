# C2 / C5 stream-count check and C3 default after the level schedule
set -e
mkdir -p gpurun_out
for s in 2 4; do
  VP9HIP_STREAMS=$s timeout -k 10 300 python bench.py --config C2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c2s_$s.json 2> gpurun_out/c2s_$s.err
  echo "C2 streams=$s $(python -c "import json;d=json.loads(open('gpurun_out/c2s_$s.json').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d['config'].get('streams_per_gpu'), d['roofline']['kernel_ms'])")"
done
timeout -k 10 400 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5.json 2> gpurun_out/c5.err
echo "C5 $(python -c "import json;d=json.loads(open('gpurun_out/c5.json').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d['config'].get('streams_per_gpu'), d['roofline']['kernel_ms'])")"
