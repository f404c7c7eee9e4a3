# frame-group streams 2 vs 3 on the other configs, and C3 again
set -e
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 300 "$@" > gpurun_out/r02ah_$tag.json 2> gpurun_out/r02ah_$tag.err; python -c "import json,sys;d=json.loads(open('gpurun_out/r02ah_$tag.json').read().strip().split(chr(10))[-1]);print('$tag', d['value'], d['ms_per_step'], d['verified_frames'])"; }
VP9HIP_STREAMS=2 run C3s2 python bench.py --no-cpu-baseline --steps 10
run C3s3 python bench.py --no-cpu-baseline --steps 10
VP9HIP_STREAMS=2 run C4s2 python bench.py --no-cpu-baseline --steps 10 --config C4
run C4s3 python bench.py --no-cpu-baseline --steps 10 --config C4
VP9HIP_STREAMS=2 run C2s2 python bench.py --no-cpu-baseline --steps 5 --config C2
run C2s3 python bench.py --no-cpu-baseline --steps 5 --config C2
