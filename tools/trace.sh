# Kernel trace of a short default bench run (timeline analysis: tools/timeline.py).
set -e
ROOT=$(pwd)
mkdir -p gpurun_out/trace_$1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $ROOT/gpurun_out/trace_$1 -o run --output-format csv -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $ROOT/gpurun_out/trace_$1.log 2>&1
echo done
