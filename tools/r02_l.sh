set -e
mkdir -p gpurun_out
timeout -k 10 300 python tools/e2e_trace.py > gpurun_out/r02l_e2e.log 2>&1
python - <<'PY'
import re
L = open("gpurun_out/r02l_e2e.log").read().splitlines()
st = [tuple(map(float, re.findall(r"setup ([\d.]+) upload ([\d.]+)", l)[0])) for l in L if "stage (device plan)" in l]
pl = [float(re.findall(r"([\d.]+) ms host wall", l)[0]) for l in L if "plan (device)" in l]
n = len(st)
print("batches", n, "setup avg %.2f ms upload avg %.2f ms plan wall avg %.2f ms" % (sum(a for a, b in st) / n, sum(b for a, b in st) / n, sum(pl) / len(pl)))
print([l for l in L if l.startswith("frames")])
PY
