# A/B switches stay bit-exact (tests/test_gpu_variants.py) + full GPU suite
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_variants.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02ad_var.log 2>&1 || { tail -40 gpurun_out/r02ad_var.log; exit 1; }
tail -8 gpurun_out/r02ad_var.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02ad_tests.log 2>&1 || { tail -40 gpurun_out/r02ad_tests.log; exit 1; }
tail -1 gpurun_out/r02ad_tests.log
