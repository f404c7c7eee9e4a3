# SQ counters of the planner with and without pass building (VP9HIP_PLAN_DBG=2)
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
export VP9HIP_PLAN_ONLY=1
for d in 0 2; do
  OUT=$ROOT/gpurun_out/plan_pmc2_$d
  mkdir -p "$OUT"
  VP9HIP_PLAN_DBG=$d timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d "$OUT/sq" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/sq.log" 2>&1
  VP9HIP_PLAN_DBG=$d timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS -d "$OUT/lds" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/lds.log" 2>&1
  echo "== dbg $d"
  python3 "$ROOT/tools/pmc_summary.py" "$OUT" | grep -A 14 "^k_plan$"
done
