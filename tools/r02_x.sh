# round-2 final evidence: GPU suite, default bench (C3, CPU legs), C2 / C4 / C5 lines with CPU
# legs, rocprofv3 trace + PMC passes of the default C3 bench
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02x_tests.log 2>&1 || { tail -40 gpurun_out/r02x_tests.log; exit 1; }
tail -1 gpurun_out/r02x_tests.log
line() { python -c "import json;d=json.loads(open('$1').read().strip().split(chr(10))[-1]);print('$2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('all_kernels_frac'), d['cpu_baseline'] and d['cpu_baseline']['value'], d.get('verified_frames'))"; }
t0=$(date +%s.%N)
timeout -k 10 400 python bench.py > gpurun_out/r02x_default.json 2> gpurun_out/r02x_default.err
t1=$(date +%s.%N)
line gpurun_out/r02x_default.json default_C3
python -c "print('default bench wall s', round($t1 - $t0, 1))"
for c in C2 C4 C5; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/r02x_$c.json 2> gpurun_out/r02x_$c.err
  line gpurun_out/r02x_$c.json $c
done
bash tools/profile.sh r02h
find gpurun_out/prof_r02h/trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_r02h/kernel_stats.csv \;
python3 tools/pmc_summary.py gpurun_out/prof_r02h > gpurun_out/prof_r02h/pmc_summary.txt
python3 tools/traffic.py gpurun_out/prof_r02h gpurun_out/prof_r02h/traffic.json > /dev/null
head -12 gpurun_out/prof_r02h/kernel_stats.csv | cut -c1-160
