# the driver's round-end sequence: GPU tests, smoke, default bench; then C2 / C4 / C5 lines with CPU legs
set -e
mkdir -p gpurun_out




start=$(date +%s); timeout -k 10 600 python bench.py > gpurun_out/r02j_default.json 2> gpurun_out/r02j_default.err
tail -1 gpurun_out/r02j_default.json
echo "default bench wall $(( $(date +%s) - start )) s"
for c in C2 C4 C5; do
  timeout -k 10 600 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 6 > gpurun_out/r02j_$c.json 2> gpurun_out/r02j_$c.err
  python -c "import json;d=json.loads(open('gpurun_out/r02j_$c.json').read().strip().split(chr(10))[-1]);print('$c', d['value'], d['ms_per_step'], d['verified_frames'], [(l['leg'], l['value'], l['cores']) for l in d['cpu_baseline']['legs']])"
done
