# GPU suite + C3 / C2 / C5 with 1 and 2 batch slots in flight
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02h_tests.log 2>&1 || { tail -40 gpurun_out/r02h_tests.log; exit 1; }
tail -1 gpurun_out/r02h_tests.log
line() { python -c "import json;d=json.loads(open('$1').read().strip().split(chr(10))[-1]);print('$2', d['value'], d['ms_per_step'], d['verify']['mismatched'] if d['verify'] else '', d['roofline']['kernel_ms'])"; }
for c in C3 C2 C5; do
  for i in 1 2; do
    timeout -k 10 300 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline --inflight $i > gpurun_out/r02h_${c}_$i.json 2> gpurun_out/r02h_${c}_$i.err
    line gpurun_out/r02h_${c}_$i.json ${c}_inflight$i
  done
done
