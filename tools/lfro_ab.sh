# k_lfro parity (C2 / C5 shapes, LF variants, GOP parity) + C2 / C5 bench lines + wave-role profile / timeline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_baseline_shapes.py tests/test_gpu_variants.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lfro_tests.log 2>&1 || { tail -30 gpurun_out/lfro_tests.log; exit 1; }
tail -2 gpurun_out/lfro_tests.log
bash tools/r04_bench.sh lfro C2 C5 && bash tools/lfro_prof.sh
