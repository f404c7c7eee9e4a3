#!/bin/bash
# round-3 end-of-round bench lines (every CPU / e2e / hwaccel leg), default C3 first
mkdir -p gpurun_out/r03k
timeout -k 10 500 python bench.py > gpurun_out/r03k/bench_default_C3.json 2> gpurun_out/r03k/bench_default_C3.err || exit 1
echo c3 done
for c in C2 C4 C5; do
  st=20; [ $c = C5 ] && st=6
  timeout -k 10 600 python bench.py --config $c --steps $st --warmup 2 > gpurun_out/r03k/bench_$c.json 2> gpurun_out/r03k/bench_$c.err || exit 1
  echo $c done
done
