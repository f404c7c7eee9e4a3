# C2 default (2 batches in flight now) and C5 default, with CPU legs and verification
set -e
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 400 "$@" > gpurun_out/r02al_$tag.json 2> gpurun_out/r02al_$tag.err; python -c "import json,sys;d=json.loads(open('gpurun_out/r02al_$tag.json').read().strip().split(chr(10))[-1]);print('$tag', d['value'], d['ms_per_step'], d['verified_frames'], d['config']['batches_in_flight'], d['config']['streams_per_gpu'])"; }
run C2 python bench.py --config C2
run C4 python bench.py --config C4
run C5 python bench.py --config C5
