# final check of the committed tree: GPU suite, smoke(), default bench
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02af_tests.log 2>&1 || { tail -40 gpurun_out/r02af_tests.log; exit 1; }
tail -1 gpurun_out/r02af_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
timeout -k 10 400 python bench.py > gpurun_out/r02af_default.json 2> gpurun_out/r02af_default.err
python -c "import json;d=json.loads(open('gpurun_out/r02af_default.json').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['verified_frames'], d['cpu_baseline']['value'])"
