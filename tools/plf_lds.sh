# k_plf LDS bank conflicts per ablation (profiling only; VP9HIP_DEBUG bits: 1 no intra
# passes, 8 no predictor rows, 16 no edge writes, 1 << 16 no LF passes), one --pmc pass each
set -e
ROOT=$(pwd); O=$ROOT/gpurun_out/plf_lds; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for d in ${DBGS:-0 1 8 16 65536}; do
  VP9HIP_DEBUG=$d timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS \
    -d $O/d$d -o run --output-format csv -- python3 $ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --verify-frames 0 > $O/d$d.log 2>&1
  python3 $ROOT/tools/pmc_summary.py $O/d$d > $O/d$d.txt
  echo "dbg=$d"; grep -A4 "^k_plf\|^k_psb\|^k_plan<\|^k_plan$" $O/d$d.txt | grep -v INSTS_LDS || true
done
