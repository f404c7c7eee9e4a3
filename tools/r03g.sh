#!/bin/bash
# round-3 inter-config run: full C5 / C2 bench lines and a C5 kernel trace of the timed steps
mkdir -p gpurun_out/r03g
timeout -k 10 500 python bench.py --config C5 --steps 6 --warmup 2 > gpurun_out/r03g/bench_C5.json 2> gpurun_out/r03g/bench_C5.err || exit 1
echo c5 done
timeout -k 10 400 python bench.py --config C2 --steps 20 --warmup 5 > gpurun_out/r03g/bench_C2.json 2> gpurun_out/r03g/bench_C2.err || exit 1
echo c2 done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03g/trace_C5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config C5 --steps 4 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r03g/trace_C5.log 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/timeline.py $GRAFT_REPO_ROOT/gpurun_out/r03g/trace_C5 0 > $GRAFT_REPO_ROOT/gpurun_out/r03g/timeline_C5.txt
cat $GRAFT_REPO_ROOT/gpurun_out/r03g/timeline_C5.txt
