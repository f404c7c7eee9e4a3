# k_lfro parity (C2 / C5 shapes, LF variants) + wave-role profile + C2 / C5 bench lines k_lfro vs k_lfrd
set -o pipefail
mkdir -p gpurun_out
VP9HIP_LFRO=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_baseline_shapes.py tests/test_gpu_variants.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lfro_tests.log 2>&1 || { tail -30 gpurun_out/lfro_tests.log; exit 1; }
tail -2 gpurun_out/lfro_tests.log
VP9HIP_LFRO=1 bash tools/r04_bench.sh lfro1 C2 C5 && VP9HIP_LFRO=0 bash tools/r04_bench.sh lfro0 C2 C5 && bash tools/lfro_prof.sh
