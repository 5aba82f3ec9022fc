#!/bin/bash
# Round-6 evidence on the current tree: GPU suite + smoke, the default bench
# (CPU baseline, front-end legs, full-size partition checks and the other
# BASELINE configs as legs), a kernel trace of the default bench, and PMC
# passes (one counter group per rocprofv3 run) of a 1-step bench.  Each GPU
# step bounded; stops at the first failure.
#   TAG=r6_final [SKIP_TESTS=1] [SKIP_BENCH=1] [SKIP_KT=1] [SKIP_PMC=1] tools/r6_final.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r6_final}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -rs -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 900 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', round(d['ms_per_step'],1), 'ms/step', round(d['value']/1e9,2), 'G tok/s', d['cpu_baseline'].get('sample_check'))"
fi
B="bench.py --no-cpu-baseline --parquet-parts 0 --frontend-mb 0 --frontend-c2-mb 0 --legs none"
if [ -z "$SKIP_KT" ]; then
# packer phase stamps (the diagnostic instantiation; s_memtime ticks summed over the waves)
LDDL_PACK_DEBUG=1 timeout -k 10 300 python -u $B --steps 1 --warmup 0 --no-sample-check > $OUT/stamps.log 2>&1 || { echo "stamps failed"; tail -5 $OUT/stamps.log; exit 1; }
grep "pack dbg" $OUT/stamps.log | head -1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python -u $B --steps 2 --warmup 1 > $OUT/kt.log 2>&1 || { echo "kernel trace failed"; tail -20 $OUT/kt.log; exit 1; }
f=$(find $OUT/kt -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats.csv
fi
[ -n "$SKIP_PMC" ] && exit 0
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
G2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"
G3="FETCH_SIZE"
G4="WRITE_SIZE"
G5="GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_SCA"
G6="TCC_HIT_sum TCC_MISS_sum"
i=0
for G in "$G1" "$G2" "$G3" "$G4" "$G5" "$G6"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $G -d $OUT/p$i -o pmc --output-format csv -- python -u $B --steps 1 --warmup 0 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt; grep -A3 'scan_kernel' $OUT/pmc_summary.txt | head -8
