set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/x_$tag.json 2> gpurun_out/x_$tag.err; python -c "import json;d=json.loads(open('gpurun_out/x_$tag.json').read().strip().split(chr(10))[-1]);print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; }
run ovl0 VP9HIP_LF_OVERLAP=0
run ovl1 VP9HIP_LF_OVERLAP=1
run ovl1_q8 VP9HIP_LF_OVERLAP=1 GPU_MAX_HW_QUEUES=8
run ovl1_s4_q8 VP9HIP_LF_OVERLAP=1 VP9HIP_STREAMS=4 GPU_MAX_HW_QUEUES=8
run ovl0_s4_q8 VP9HIP_LF_OVERLAP=0 VP9HIP_STREAMS=4 GPU_MAX_HW_QUEUES=8
run ovl1_s6_q16 VP9HIP_LF_OVERLAP=1 VP9HIP_STREAMS=6 GPU_MAX_HW_QUEUES=16
run ovl1_s2 VP9HIP_LF_OVERLAP=1 VP9HIP_STREAMS=2
