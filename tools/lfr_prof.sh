# k_lfr phase breakdown at C5 / C2 (LFR_PROF build swapped in on the box only)
set -e
mkdir -p gpurun_out
cp ffmpeg-hybrid_amd/prof/libvp9hip.so ffmpeg-hybrid_amd/libvp9hip.so
for c in C5 C2; do
  timeout -k 10 300 python tools/lfr_prof.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/lfrprof_$c.json 2> gpurun_out/lfrprof_$c.err
  echo $c; tail -14 gpurun_out/lfrprof_$c.err
done
