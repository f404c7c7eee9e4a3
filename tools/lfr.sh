# k_lfr check: GPU parity, then C3 / C2 benches: row-pipelined LF (prefetch off / on) and diagonal launches.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lfr_tests.log 2>&1 || { tail -40 gpurun_out/lfr_tests.log; exit 1; }
tail -1 gpurun_out/lfr_tests.log
for cfg in ${CFGS:-C3 C2}; do
  for m in ${MODES:-1:0 1:1 0:0}; do
    VP9HIP_LFROW=${m%%:*} VP9HIP_LFR_PF=${m##*:} timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/lfr_${cfg}_$m.json 2> gpurun_out/lfr_${cfg}_$m.err
    echo "$cfg lfrow:pf=$m $(python -c "import json;d=json.loads(open('gpurun_out/lfr_${cfg}_$m.json').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['kernel_ms'])")"
  done
done
