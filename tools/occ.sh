set -e
mkdir -p gpurun_out
for pad in ${PADS:-0 5 11 24 37}; do
  d=$(( pad * 256 ))
  VP9HIP_STREAMS=1 VP9HIP_DEBUG=$d timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/occ_$pad.log 2>&1
  echo "pad=${pad}KB $(python -c "import json;d=json.loads(open('gpurun_out/occ_$pad.log').read().strip().split(chr(10))[-1]);print(d['roofline']['kernel_ms'])")"
done
