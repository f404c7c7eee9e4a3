# sweep after the 2-stream default: C3 at 1 stream, C2 with 2 batches in flight
set -e
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 300 "$@" > gpurun_out/r02ak_$tag.json 2> gpurun_out/r02ak_$tag.err; python -c "import json,sys;d=json.loads(open('gpurun_out/r02ak_$tag.json').read().strip().split(chr(10))[-1]);print('$tag', d['value'], d['ms_per_step'], d['verified_frames'])"; }
VP9HIP_STREAMS=1 run C3s1 python bench.py --no-cpu-baseline --steps 10
run C3 python bench.py --no-cpu-baseline --steps 10
run C2if1 python bench.py --no-cpu-baseline --steps 5 --config C2
run C2if2 python bench.py --no-cpu-baseline --steps 5 --config C2 --inflight 2
