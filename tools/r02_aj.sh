# rocprofv3 kernel trace + stats (csv) of the default bench workload, 2 frame-group streams
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02aj_prof -o run -- python bench.py --no-cpu-baseline --steps 5 > gpurun_out/r02aj_prof.log 2>&1
find gpurun_out/r02aj_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r02aj_kernel_stats.csv \;
find gpurun_out/r02aj_prof -name "*kernel_trace.csv" -delete
head -12 gpurun_out/r02aj_kernel_stats.csv | cut -d, -f1-6
