#!/bin/bash
# GPU suite (log under gpurun_out/check), then optional profiles. usage: tools/r04_check.sh [prof args...]
set -o pipefail
O=gpurun_out/check; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
