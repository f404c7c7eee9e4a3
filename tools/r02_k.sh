# GPU suite, then the default bench (e2e decoder with alternating batch slots)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02k_tests.log 2>&1 || { tail -40 gpurun_out/r02k_tests.log; exit 1; }
tail -1 gpurun_out/r02k_tests.log
timeout -k 10 600 python bench.py > gpurun_out/r02k_default.json 2> gpurun_out/r02k_default.err
python -c "import json;d=json.loads(open('gpurun_out/r02k_default.json').read().strip().split(chr(10))[-1]);print(d['value'], d['verified_frames'], d['e2e_decoder']['fps'], d['e2e_decoder']['low_rate']['fps'], d['e2e_decoder']['low_rate']['host_parse'])"
