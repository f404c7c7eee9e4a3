# Quick check: GPU parity, then C3 bench at the default stream count and single-stream kernel times.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
for s in default 1; do
  if [ $s = default ]; then unset VP9HIP_STREAMS; else export VP9HIP_STREAMS=$s; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/q_$s.json 2> gpurun_out/q_$s.err
  echo "streams=$s $(python -c "import json;d=json.loads(open('gpurun_out/q_$s.json').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d['config']['streams_per_gpu'], d['roofline']['kernel_ms'])")"
done
