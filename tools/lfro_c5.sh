# C5 k_lfro vs k_lfrd: default streams ABAB, then one frame-group stream (no chain overlap)
set -o pipefail
VP9HIP_LFRO=1 bash tools/r04_bench.sh c5a1 C5 && VP9HIP_LFRO=0 bash tools/r04_bench.sh c5a0 C5 && \
VP9HIP_LFRO=1 bash tools/r04_bench.sh c5b1 C5 && VP9HIP_LFRO=0 bash tools/r04_bench.sh c5b0 C5 && \
VP9HIP_STREAMS=1 VP9HIP_LFRO=1 bash tools/r04_bench.sh c5s1 C5 && VP9HIP_STREAMS=1 VP9HIP_LFRO=0 bash tools/r04_bench.sh c5s0 C5
