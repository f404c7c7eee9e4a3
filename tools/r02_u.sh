# C3 / C4 with the row-pipelined LF (k_lfrd) for wide keyframe phases too (VP9HIP_LFROW=2)
set -e
mkdir -p gpurun_out
line() { python -c "import json;d=json.loads(open('$1').read().strip().split(chr(10))[-1]);print('$2', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'), d.get('verified_frames'))"; }
for c in C3 C4; do
  timeout -k 10 300 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r02u_$c.json 2> gpurun_out/r02u_$c.err
  line gpurun_out/r02u_$c.json $c
  VP9HIP_LFROW=2 timeout -k 10 300 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r02u_${c}_lfrow.json 2> gpurun_out/r02u_${c}_lfrow.err
  line gpurun_out/r02u_${c}_lfrow.json ${c}_lfrow2
done
