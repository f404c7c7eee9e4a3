#!/bin/bash
# GPU suite, then (optional) a build A/B (tools/abso.sh) and the rocprofv3 passes of the
# default C3 bench (tools/profile.sh TAG). usage: tools/gpu_check.sh [TAG] [ab rounds]
set -o pipefail
O=gpurun_out/check; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
if [ -n "$2" ] && [ -f ffmpeg-hybrid_amd/ab_base/libvp9hip.so ]; then bash tools/abso.sh $2 || exit 1; fi
if [ -n "$1" ]; then bash tools/profile.sh $1 || exit 1; fi
