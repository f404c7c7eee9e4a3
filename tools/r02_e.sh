# GPU suite + default bench (serialised timing steps)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02e_tests.log 2>&1 || { tail -40 gpurun_out/r02e_tests.log; exit 1; }
tail -1 gpurun_out/r02e_tests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02e_C3.json 2> gpurun_out/r02e_C3.err
tail -1 gpurun_out/r02e_C3.json
