# final check with 2 frame-group streams by default: GPU suite, smoke(), default bench, kernel trace
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02ai_tests.log 2>&1 || { tail -40 gpurun_out/r02ai_tests.log; exit 1; }
tail -1 gpurun_out/r02ai_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
timeout -k 10 400 python bench.py > gpurun_out/r02ai_default.json 2> gpurun_out/r02ai_default.err
python -c "import json;d=json.loads(open('gpurun_out/r02ai_default.json').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['verified_frames'], d['cpu_baseline']['value'])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02ai_prof -o run -- python bench.py --no-cpu-baseline --steps 5 > gpurun_out/r02ai_prof.log 2>&1
find gpurun_out/r02ai_prof -name "*kernel_stats.csv" | head -3
