#!/bin/bash
# rocprofv3 trace + PMC passes (tools/profile.sh) for several configs. usage: tools/prof_cfgs.sh TAG CFG...
set -o pipefail
TAG=$1; shift
for c in "$@"; do
  st=3; [ $c = C5 ] && st=2
  bash tools/profile.sh ${TAG}_$c --config $c --steps $st --warmup 1 --no-cpu-baseline || exit 1
done
