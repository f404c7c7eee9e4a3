# k_mc 8 rows per lane (MC_ROWS8=1, default) vs 4 (prof/ build with MC_ROWS8=0): GPU suite + C5 / C4
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02w_tests.log 2>&1 || { tail -40 gpurun_out/r02w_tests.log; exit 1; }
tail -1 gpurun_out/r02w_tests.log
line() { python -c "import json;d=json.loads(open('$1').read().strip().split(chr(10))[-1]);print('$2', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'), d.get('verified_frames'))"; }
timeout -k 10 300 python bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02w_C5.json 2> gpurun_out/r02w_C5.err
line gpurun_out/r02w_C5.json C5_rows8
cp ffmpeg-hybrid_amd/prof/libvp9hip.so ffmpeg-hybrid_amd/libvp9hip.so
timeout -k 10 300 python bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02w_C5_r4.json 2> gpurun_out/r02w_C5_r4.err
line gpurun_out/r02w_C5_r4.json C5_rows4
