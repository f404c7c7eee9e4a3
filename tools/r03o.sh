set -o pipefail
mkdir -p gpurun_out/r03o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03o/tests.log 2>&1 || { tail -30 gpurun_out/r03o/tests.log; exit 1; }
tail -1 gpurun_out/r03o/tests.log
bash tools/abso.sh 2
