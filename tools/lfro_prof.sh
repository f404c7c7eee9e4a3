# k_lfro wave-role breakdown at C5 / C2 (LFR_PROF build swapped in on the box only)
set -e
mkdir -p gpurun_out
cp ffmpeg-hybrid_amd/prof/libvp9hip.so ffmpeg-hybrid_amd/libvp9hip.so
for c in C5 C2; do
  timeout -k 10 300 python tools/lfro_prof.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/lfroprof_$c.json 2> gpurun_out/lfroprof_$c.err
  echo $c; tail -40 gpurun_out/lfroprof_$c.err
done
