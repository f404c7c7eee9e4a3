# round 3: N batch slots -- GPU suite, then batches-in-flight A/B per config (no CPU legs)
set -o pipefail
O=gpurun_out/r03m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in C3 C5 C2; do
  for n in 2 3 4; do
    timeout -k 10 300 python bench.py --config $cfg --inflight $n --steps 8 --warmup 2 --no-cpu-baseline --verify-frames 4 > $O/${cfg}_if$n.json 2> $O/${cfg}_if$n.err || { echo "$cfg $n failed"; tail -5 $O/${cfg}_if$n.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/${cfg}_if$n.json').read().strip().split(chr(10))[-1]);print('$cfg', $n, d['value'], d['ms_per_step'], d['verify']['frames'], d['verify']['of'], len(d['verify']['mismatched']))"
  done
done
