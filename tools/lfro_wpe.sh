# k_lfro at 4 waves / EU (2 workgroups per CU at high bit depth): C5 parity (variants, shapes) + C5 / C2 lines
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_baseline_shapes.py tests/test_gpu_variants.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lfro_tests.log 2>&1 || { tail -30 gpurun_out/lfro_tests.log; exit 1; }
tail -1 gpurun_out/lfro_tests.log
bash tools/r04_bench.sh wpe4 C5 C2 && BARGS="--inflight 3" bash tools/c5_conc.sh 2>/dev/null | head -0; true
