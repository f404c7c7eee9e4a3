set -o pipefail
mkdir -p gpurun_out/r03l
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03l/tests.log 2>&1 || { tail -30 gpurun_out/r03l/tests.log; exit 1; }
tail -2 gpurun_out/r03l/tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03l/bench.json 2> gpurun_out/r03l/bench.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/r03l/bench.json').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d['verify']['frames'], d['roofline']['frac'], d['roofline']['avg_launch_us'])"
VP9HIP_STATIC=0 VP9HIP_PLAN_PROF=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03l/pprof.json 2> gpurun_out/r03l/pprof.err || exit 1
grep "plan phases" gpurun_out/r03l/pprof.err | tail -2
