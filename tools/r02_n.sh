# k_plan ablations (timing only; frames are wrong, so the bench's verification fails: ignored)
mkdir -p gpurun_out
for d in 0 2; do
  VP9HIP_PLAN_DBG=$d timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abl_plan_$d.json 2> gpurun_out/abl_plan_$d.err
  python -c "import json;d=json.loads(open('gpurun_out/abl_plan_$d.json').read().strip().split(chr(10))[-1]);print('dbg $d', d['roofline']['kernel_ms']['k_plan'])"
done
