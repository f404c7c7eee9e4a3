#!/bin/bash
# Round-6 evidence on one box: GPU suite, the serialised-step profile of the default C3 bench
# (tools/profile.sh TAG, copied to profiles/TAG/C3 so the bench lines below cite it), then the
# default bench line and the other configs (tools/round_bench.sh). usage: tools/final_r06.sh TAG
set -o pipefail
T=${1:?tag}
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
tail -1 gpurun_out/${T}_tests.log
grep -q " passed" gpurun_out/${T}_tests.log && ! grep -q "failed" gpurun_out/${T}_tests.log || exit 1
bash tools/profile.sh $T || exit 1
mkdir -p profiles/$T/C3
cp gpurun_out/prof_$T/trace/run_kernel_stats.csv profiles/$T/C3/kernel_stats.csv
cp gpurun_out/prof_$T/pmc_summary.txt gpurun_out/prof_$T/traffic.json profiles/$T/C3/
bash tools/round_bench.sh $T
