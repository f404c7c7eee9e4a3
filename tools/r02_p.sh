# double-buffered k_lfr (k_lfrd): GPU suite, C5 / C2 / C3 lines, A/B vs k_lfr, phase profile
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02p_tests.log 2>&1 || { tail -40 gpurun_out/r02p_tests.log; exit 1; }
tail -1 gpurun_out/r02p_tests.log
line() { python -c "import json;d=json.loads(open('$1').read().strip().split(chr(10))[-1]);print('$2', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'), d.get('verified_frames'))"; }
for c in C5 C2; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02p_$c.json 2> gpurun_out/r02p_$c.err
  line gpurun_out/r02p_$c.json $c
  VP9HIP_LFR_DB=0 timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02p_${c}_old.json 2> gpurun_out/r02p_${c}_old.err
  line gpurun_out/r02p_${c}_old.json ${c}_old
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02p_C3.json 2> gpurun_out/r02p_C3.err
line gpurun_out/r02p_C3.json C3
cp ffmpeg-hybrid_amd/prof/libvp9hip.so ffmpeg-hybrid_amd/libvp9hip.so
for c in C5 C2; do
  timeout -k 10 300 python tools/lfr_prof.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/lfrprof2_$c.json 2> gpurun_out/lfrprof2_$c.err
  echo $c; tail -15 gpurun_out/lfrprof2_$c.err
done
