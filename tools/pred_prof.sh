# intra workgroup phase breakdown at C3 / C2 (PRED_PROF build swapped in on the box only)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_baseline_shapes.py -x -q --timeout 300 --timeout-method thread > gpurun_out/predprof_tests.log 2>&1 || { tail -30 gpurun_out/predprof_tests.log; exit 1; }
tail -1 gpurun_out/predprof_tests.log
cp ffmpeg-hybrid_amd/prof/libvp9hip.so ffmpeg-hybrid_amd/libvp9hip.so
for c in ${CFGS:-C3 C2}; do
  timeout -k 10 300 python tools/pred_prof.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/predprof_$c.json 2> gpurun_out/predprof_$c.err
  echo $c; tail -8 gpurun_out/predprof_$c.err
done
