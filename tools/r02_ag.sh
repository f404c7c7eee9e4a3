# knob sweep on the rebuilt tree (C3): frame-group streams, batches in flight
set -e
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 300 "$@" > gpurun_out/r02ag_$tag.json 2> gpurun_out/r02ag_$tag.err; python -c "import json,sys;d=json.loads(open('gpurun_out/r02ag_$tag.json').read().strip().split(chr(10))[-1]);print('$tag', d['value'], d['ms_per_step'], d['verified_frames'])"; }
run def python bench.py --no-cpu-baseline --steps 10
VP9HIP_STREAMS=2 run s2 python bench.py --no-cpu-baseline --steps 10
VP9HIP_STREAMS=4 run s4 python bench.py --no-cpu-baseline --steps 10
run if1 python bench.py --no-cpu-baseline --steps 10 --inflight 1
run def2 python bench.py --no-cpu-baseline --steps 10
