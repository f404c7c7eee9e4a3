#!/bin/bash
# Timing-only ablations of the pixel kernels (VP9HIP_DEBUG bits skip work; the frames are then
# wrong and the bench's verification is off): fps, ms per step and the serialised kernel ms.
# intra (k_pred / k_plf intra waves): 1 passes, 2 interior stores, 4 tile loads (the per-pass
# ablations 8 pass rows / 16 pass edges are a build flag: make PROF=-DPRED_ABL=8 prof, and
# ../prof/libvp9hip.so copied over the library on the GPU box, as tools/pred_prof.sh does);
# loop filter (bits << 16): 1 filter passes, 2 stores, 4 loads.
# usage: DBGS="0 1 2 ..." [BARGS=...] tools/ablate.sh TAG
set -o pipefail
O=gpurun_out/ablate_${1:-x}; mkdir -p $O
for d in ${DBGS:-0 1 2 4 65536 131072 262144}; do
  VP9HIP_DEBUG=$d timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --verify-frames 0 ${BARGS:-} > $O/dbg_$d.json 2> $O/dbg_$d.err || { echo "dbg=$d failed"; tail -3 $O/dbg_$d.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/dbg_$d.json').read().strip().split(chr(10))[-1]);km=d['roofline']['kernel_ms'];print('dbg=$d', d['value'], d['ms_per_step'], {k: v for k, v in km.items() if v})"
done
