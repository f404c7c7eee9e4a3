#!/bin/bash
# VP9HIP_MCR=1 (a level phase's residuals one chain position early, added by k_mcq from the
# residual planes) against the default: GPU parity of the inter shapes with it on, then bench
# lines alternated on the same box. usage: tools/mcr_ab.sh TAG [configs]
set -o pipefail
O=gpurun_out/mcr_${1:-x}; mkdir -p $O
VP9HIP_MCR=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_baseline_shapes.py tests/test_gpu_variants.py tests/test_gpu_parity.py tests/test_gpu_streams.py \
  tests/test_ivf_decoder.py tests/test_gpu_rejected_batch.py > $O/parity.txt 2>&1 \
  || { echo "parity failed"; tail -30 $O/parity.txt; exit 1; }
tail -1 $O/parity.txt
line() { python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]);km=d['roofline']['kernel_ms'];print(sys.argv[2], d['value'], d['ms_per_step'], d.get('verified_frames'), {k: v for k, v in km.items() if v})" "$@"; }
for cfg in ${2:-C2 C5}; do
  case $cfg in C5) B="--steps 6 --warmup 2";; *) B="--steps 20";; esac
  for rep in 1 2; do
    for m in 0 1; do
      VP9HIP_MCR=$m timeout -k 10 240 python bench.py --config $cfg $B --no-cpu-baseline > $O/${cfg}_m${m}_$rep.json 2> $O/${cfg}_m${m}_$rep.err \
        || { echo "$cfg mcr=$m failed"; tail -3 $O/${cfg}_m${m}_$rep.err; exit 1; }
      line $O/${cfg}_m${m}_$rep.json "$cfg mcr=$m rep=$rep"
    done
  done
done
