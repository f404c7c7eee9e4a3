#!/bin/bash
# rocprofv3 passes over a reduced bench run (GPU box). Usage: tools/profile.sh TAG [bench args]
# 1) kernel trace + stats, 2-4) PMC passes (separate runs: SQ timing/instruction mix,
# FETCH_SIZE, WRITE_SIZE), as MI355X_MICROARCH.md's rocprofv3 section prescribes.
set -e
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
ARGS=${*:-"--serial-only --steps 10 --warmup 2"}    # the bench workload (C3, 120 frames): its serialised timing steps
cd /tmp && export TMPDIR=/tmp
run() { local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python3 "$ROOT/bench.py" $ARGS > "$OUT/$name.log" 2>&1
  echo "[profile] $name done"; }
run trace --kernel-trace --stats
run sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU
run lds --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
python3 "$ROOT/tools/traffic.py" "$OUT" "$OUT/traffic.json" > /dev/null
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/pmc_summary.txt"
echo "[profile] summaries written"

