# rocprofv3 kernel trace + PMC passes (SQ, LDS, FETCH, WRITE) of the C5 and C2 benches with k_lfrd
set -e
mkdir -p gpurun_out
for c in C5 C2; do
  bash tools/profile.sh r02g_$c --config $c --steps 2 --warmup 1 --no-cpu-baseline
  find gpurun_out/prof_r02g_$c/trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_r02g_$c/kernel_stats.csv \;
  python3 tools/pmc_summary.py gpurun_out/prof_r02g_$c > gpurun_out/prof_r02g_$c/pmc_summary.txt
  python3 tools/traffic.py gpurun_out/prof_r02g_$c gpurun_out/prof_r02g_$c/traffic.json > /dev/null
  grep -i "lfr" gpurun_out/prof_r02g_$c/kernel_stats.csv | head -3
  grep -i -A12 "k_lfr" gpurun_out/prof_r02g_$c/pmc_summary.txt | head -14
done
