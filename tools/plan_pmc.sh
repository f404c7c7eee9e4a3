# PMC passes over the device planner alone (VP9HIP_PLAN_ONLY=1: run_batch stops after planning)
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/plan_pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export VP9HIP_PLAN_ONLY=1
run() { local name=$1; shift
  timeout -s KILL 120 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/$name.log" 2>&1
  echo "[pmc] $name rc=$?"; }
run trace --kernel-trace --stats
run sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
run lds --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SMEM
python3 "$ROOT/tools/pmc_summary.py" "$OUT"
