# GPU parity, then the default bench (as the driver runs it) and C2 / C5 quick lines,
# device planner (default) vs the host planner (VP9HIP_HOST_PLAN=1).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_tests.log 2>&1 || { tail -40 gpurun_out/r02_tests.log; exit 1; }
tail -1 gpurun_out/r02_tests.log
timeout -k 10 500 python bench.py > gpurun_out/r02_default.json 2> gpurun_out/r02_default.err
tail -1 gpurun_out/r02_default.json
line() { python -c "import json;d=json.loads(open('$1').read().strip().split(chr(10))[-1]);print('$2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; }
for c in ${CFGS:-C2 C5}; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02_$c.json 2> gpurun_out/r02_$c.err
  line gpurun_out/r02_$c.json $c
done
VP9HIP_HOST_PLAN=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02_hostplan.json 2> gpurun_out/r02_hostplan.err
line gpurun_out/r02_hostplan.json C3_hostplan
