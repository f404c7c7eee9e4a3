# k_mcq parity (MC tests, subsampling, variants, C2/C5 shapes), then C2 / C5 bench lines: k_mcq default, k_mcq 1 slice, k_mcp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_subsampling.py tests/test_gpu_variants.py tests/test_gpu_baseline_shapes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mcq_tests.log 2>&1 || { tail -40 gpurun_out/mcq_tests.log; exit 1; }
tail -2 gpurun_out/mcq_tests.log
bash tools/r04_bench.sh mcq3 C2 C5 && VP9HIP_MCQ_SLICES=1 bash tools/r04_bench.sh mcq3s1 C2 C5 && VP9HIP_MCP=2 bash tools/r04_bench.sh mcq2 C2 C5
for t in mcq3 mcq3s1 mcq2; do for c in C2 C5; do python -c "
import json;d=json.loads(open('gpurun_out/$t/bench_$c.json').read().strip().split(chr(10))[-1]);r=d['roofline']
print('$t $c', d['value'], 'k_mc us/launch', round(r['kernel_ms']['k_mc']/max(1,r['kernel_launches']['k_mc'])*1000,1))"; done; done
