# rocprofv3 kernel trace of the FFHWAccel harness (device consumer) on the C3 sample: this
# build vs ffmpeg-hybrid_amd/ab_r03 (the round-3 library), for per-kernel A/B
set -e
mkdir -p gpurun_out/hwprof
timeout -k 10 200 python tools/mk_ivf.py C3 10 gpurun_out/hwprof/c3.ivf
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/hwprof/head -o run --output-format csv -- $R/tests/c/hwaccel_harness $R/gpurun_out/hwprof/c3.ivf - 8 1 1 1 16 device 0
export LD_LIBRARY_PATH=$R/ffmpeg-hybrid_amd/ab_r03
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/hwprof/r03 -o run --output-format csv -- $R/ffmpeg-hybrid_amd/ab_r03/hwaccel_harness $R/gpurun_out/hwprof/c3.ivf - 8 1 1 1 16 device 0
rm -f $R/gpurun_out/hwprof/c3.ivf
