# round 3: hardware queues x batches in flight (no CPU legs)
set -o pipefail
O=gpurun_out/r03n; mkdir -p $O
run() {  # name config inflight [env...]
  local name=$1 cfg=$2 n=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --config $cfg --inflight $n --steps 8 --warmup 2 --no-cpu-baseline --verify-frames 4 > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$name.json').read().strip().split(chr(10))[-1]);print('$name', d['value'], d['ms_per_step'], d['verify']['frames'], d['verify']['of'], len(d['verify']['mismatched']))"
}
run C5_if4_q8 C5 4 GPU_MAX_HW_QUEUES=8
run C2_if4_q8 C2 4 GPU_MAX_HW_QUEUES=8
run C5_if4 C5 4 X=1
run C3_if2_q8 C3 2 GPU_MAX_HW_QUEUES=8
run C3_if4_q8 C3 4 GPU_MAX_HW_QUEUES=8
run C4_if2 C4 2 X=1
run C4_if4 C4 4 X=1
run C5_if4_s3 C5 4 VP9HIP_STREAMS=3
