# k_resid_multi with one-wave workgroups: GPU suite + C2 / C5
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02ac_tests.log 2>&1 || { tail -40 gpurun_out/r02ac_tests.log; exit 1; }
tail -1 gpurun_out/r02ac_tests.log
line() { python -c "import json;d=json.loads(open('$1').read().strip().split(chr(10))[-1]);print('$2', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'), d.get('verified_frames'))"; }
for c in C2 C5; do
  timeout -k 10 300 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r02ac_$c.json 2> gpurun_out/r02ac_$c.err
  line gpurun_out/r02ac_$c.json $c
done
