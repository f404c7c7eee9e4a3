# fused intra+LF launches vs separate (C3), GPU tests first
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 ${BARGS:-} > gpurun_out/x_$tag.json 2> gpurun_out/x_$tag.err; python -c "import json;d=json.loads(open('gpurun_out/x_$tag.json').read().strip().split(chr(10))[-1]);print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel'], d['roofline']['frac'])"; }
run plf0 VP9HIP_PLF=0
run plf1 VP9HIP_PLF=1
run plf1_s2 VP9HIP_PLF=1 VP9HIP_STREAMS=2
run plf1_s4 VP9HIP_PLF=1 VP9HIP_STREAMS=4
BARGS="--config C2" run c2_plf0 VP9HIP_PLF=0
BARGS="--config C2" run c2_plf1 VP9HIP_PLF=1
