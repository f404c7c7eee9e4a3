# GPU suite, then the rocprofv3 trace + PMC passes of the C3 bench (profiles/r02d)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02i_tests.log 2>&1 || { tail -40 gpurun_out/r02i_tests.log; exit 1; }
tail -1 gpurun_out/r02i_tests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02i_C3.json 2> gpurun_out/r02i_C3.err
tail -1 gpurun_out/r02i_C3.json
bash tools/profile.sh r02d
python3 tools/pmc_summary.py gpurun_out/prof_r02d > gpurun_out/prof_r02d/pmc_summary.txt
python3 tools/traffic.py gpurun_out/prof_r02d gpurun_out/prof_r02d/traffic.json
find gpurun_out/prof_r02d/trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_r02d/kernel_stats.csv \;
