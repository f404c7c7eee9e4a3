# default bench lines (CPU baseline + e2e / hwaccel legs) of the given configs
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for c in "$@"; do
  timeout -k 10 560 python -u bench.py --config $c > $O/full_$c.json 2> $O/full_$c.err || { tail -5 $O/full_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/full_$c.json').read().strip().split(chr(10))[-1]);print('$c', d['value'], json.dumps(d.get('e2e_decoder')), json.dumps(d.get('e2e_decoder',{}) and d['e2e_decoder'].get('hwaccel_path')))"
done
