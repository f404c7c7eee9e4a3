# final round-2 evidence: GPU suite, default bench (C3 with CPU legs), C2 / C4 / C5 with CPU legs,
# rocprofv3 trace + PMC of the default C3 bench and of C5 (k_lfrd)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02ab_tests.log 2>&1 || { tail -40 gpurun_out/r02ab_tests.log; exit 1; }
tail -1 gpurun_out/r02ab_tests.log
line() { python -c "import json;d=json.loads(open('$1').read().strip().split(chr(10))[-1]);print('$2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('all_kernels_frac'), d['cpu_baseline'] and d['cpu_baseline']['value'], d.get('verified_frames'))"; }
t0=$(date +%s.%N)
timeout -k 10 400 python bench.py > gpurun_out/r02ab_default.json 2> gpurun_out/r02ab_default.err
t1=$(date +%s.%N)
line gpurun_out/r02ab_default.json default_C3
python -c "print('default bench wall s', round($t1 - $t0, 1))"
for c in C2 C4 C5; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/r02ab_$c.json 2> gpurun_out/r02ab_$c.err
  line gpurun_out/r02ab_$c.json $c
done
for t in r02i r02i_C5; do
  if [ $t = r02i ]; then bash tools/profile.sh $t; else bash tools/profile.sh $t --config C5 --steps 2 --warmup 1 --no-cpu-baseline; fi
  find gpurun_out/prof_$t/trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_$t/kernel_stats.csv \;
  python3 tools/pmc_summary.py gpurun_out/prof_$t > gpurun_out/prof_$t/pmc_summary.txt
  python3 tools/traffic.py gpurun_out/prof_$t gpurun_out/prof_$t/traffic.json > /dev/null
  head -6 gpurun_out/prof_$t/kernel_stats.csv | cut -c1-150
done
