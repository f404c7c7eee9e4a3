set -o pipefail
for ns in 3 4 6; do VP9HIP_MCQ_SLICES=$ns bash tools/r04_bench.sh sl$ns C5 || exit 1; done
for ns in 4 12 16; do VP9HIP_MCQ_SLICES=$ns bash tools/r04_bench.sh sl$ns C2 || exit 1; done
for f in gpurun_out/sl*/bench_*.json; do python -c "
import json;d=json.loads(open('$f').read().strip().split(chr(10))[-1]);r=d['roofline']
print('$f', d['value'], 'k_mc us/launch', round(r['kernel_ms']['k_mc']/max(1,r['kernel_launches']['k_mc'])*1000,1))"; done
