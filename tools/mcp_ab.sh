# k_mc / k_mcp A/B on the GOP-chain configs (1-GPU bench lines, no CPU legs)
set -o pipefail
O=gpurun_out/mcp_ab; mkdir -p $O
run() { local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps $([ $cfg = C5 ] && echo 4 || echo 10) --warmup 2 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$tag.json').read().strip().split(chr(10))[-1]);r=d['roofline'];print('$tag', d['value'], round(r['kernel_ms']['k_mc']/max(1,r['kernel_launches']['k_mc'])*1000,1), 'us/k_mc launch', d['verify']['mismatched'])"; }
for a in ${RUNS:-C5:VP9HIP_MCP=1 C5:VP9HIP_MCP=0 C2:VP9HIP_MCP=1 C2:VP9HIP_MCP=2}; do run ${a/:/_} ${a%%:*} ${a#*:} || exit 1; done
