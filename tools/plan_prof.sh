# rocprofv3 kernel trace of the C3 bench (device planner): per-kernel durations.
set -e
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/plan_prof${TAG:-}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ${BARGS:-} > "$OUT/bench.log" 2>&1
find "$OUT" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
head -30 "$OUT/kernel_stats.csv"
