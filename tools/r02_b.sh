# lfr timeout tests + planner phase profile (C3, C2)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lfr_timeout.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02b_tests.log 2>&1 || { tail -40 gpurun_out/r02b_tests.log; exit 1; }
tail -3 gpurun_out/r02b_tests.log
VP9HIP_PLAN_PROF=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r02b_pp.json 2> gpurun_out/r02b_pp.err
tail -2 gpurun_out/r02b_pp.err
VP9HIP_PLAN_PROF=1 timeout -k 10 300 python bench.py --config C2 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r02b_pp2.json 2> gpurun_out/r02b_pp2.err
tail -2 gpurun_out/r02b_pp2.err
