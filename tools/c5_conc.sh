# C5 concurrency: batches in flight 1 / 2 / 3, and 8 hardware queues at 2 / 3 in flight
set -o pipefail
O=gpurun_out/c5conc; mkdir -p $O
run() { local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config C5 --steps 4 --warmup 2 --no-cpu-baseline $BARGS > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$tag.json').read().strip().split(chr(10))[-1]);print('$tag', d['value'], d['ms_per_step'], d['config'].get('batches_in_flight'))"; }
BARGS="--inflight 1" run if1 X=1 && BARGS="--inflight 2" run if2 X=1 && BARGS="--inflight 3" run if3 X=1 && \
BARGS="--inflight 2" run if2q8 GPU_MAX_HW_QUEUES=8 && BARGS="--inflight 3" run if3q8 GPU_MAX_HW_QUEUES=8 && BARGS="--inflight 4" run if4q8 GPU_MAX_HW_QUEUES=8
