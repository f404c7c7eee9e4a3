set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02m_tests.log 2>&1 || { tail -40 gpurun_out/r02m_tests.log; exit 1; }
tail -1 gpurun_out/r02m_tests.log
bash tools/r02_l.sh
