#!/bin/bash
# CPU: the host side and the FFHWAccel adapter (over tests/c/fake_device.cpp) under ASan +
# UBSan and TSan; logs into profiles/$TAG (default r04_sanitize). usage: tools/sanitize.sh [TAG]
set -o pipefail
TAG=${1:-r04_sanitize}
O=profiles/$TAG; mkdir -p $O
make -s -j8 -C ffmpeg-hybrid_amd/csrc sanitize || exit 1
python3 - <<'PY' || exit 1
import sys, importlib
sys.path.insert(0, "tests")
v9 = importlib.import_module("ffmpeg-hybrid_amd")
from test_ivf_decoder import _stream
from test_stream import _frames, encode_stream
pk = _stream(v9, 200, 130)
open("/tmp/san_s.ivf", "wb").write(v9.ivf_write(pk, 200, 130))
open("/tmp/san_s.webm", "wb").write(v9.webm_write(pk, 200, 130, lacing="xiph", voids=True))
open("/tmp/san_e.webm", "wb").write(v9.webm_write(pk, 200, 130, lacing="ebml", unknown_sizes=True, other_track=True))
# a longer GOP with 4 tile columns and backward adaptation for the adapter runs
fr = _frames(v9, 1024, 160, 24, log2_tile_cols=2)
d, _ = encode_stream(v9, fr, lambda i: dict(refresh_ctx=1, parallel=0) if i % 3 == 1 else {})
open("/tmp/san_g.ivf", "wb").write(v9.ivf_write(d, 1024, 160))
PY
B=tests/c/build
for v in asan tsan; do
  { echo "== host_san_$v 200 mutations + 3 containers"; ./$B/host_san_$v 200 /tmp/san_s.ivf /tmp/san_s.webm /tmp/san_e.webm; echo "exit $?"; } > $O/host_san_$v.log 2>&1
  for args in "2 0 download 16" "2 8 device 4" "2 3 thread 1" "2 16 thread 8" "1 0 download 0 -1"; do
    set -- $args
    { echo "== hwaccel_cpu_$v san_g.ivf passes $1 lag $2 mode $3 depth $4 ${5:+extra $5}"; ./$B/hwaccel_cpu_$v /tmp/san_g.ivf - 8 1 1 $args; echo "exit $?"; } >> $O/hwaccel_cpu_$v.log 2>&1
  done
done
grep -l "ERROR: AddressSanitizer\|WARNING: ThreadSanitizer\|runtime error" $O/*.log && { echo "sanitizer findings"; exit 1; }
grep -h "^exit" $O/*.log | sort | uniq -c
