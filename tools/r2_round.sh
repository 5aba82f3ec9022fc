#!/bin/bash
# Evidence session on the current tree: GPU tests, smoke, the default bench,
# a kernel trace of the bench and PMC passes of a 1-step bench (one counter
# group per rocprofv3 run).  Each GPU step bounded; stops at the first failure.
#   TAG=r2_final SKIP_TESTS=1 BENCH_ARGS="--corpus code" tools/r2_round.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_round}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
  cat $OUT/smoke.log
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
  tail -1 $OUT/bench.log > $OUT/bench.json
  cat $OUT/bench.json
fi
B="bench.py --no-cpu-baseline --parquet-parts 0 --frontend-mb 0 ${BENCH_ARGS}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python -u $B --steps 2 --warmup 1 > $OUT/kt.log 2>&1 || { echo "kernel trace failed"; tail -20 $OUT/kt.log; exit 1; }
f=$(find $OUT/kt -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats.csv; cut -d, -f1-4 $f | head -16
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
python tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt; head -150 $OUT/pmc_summary.txt
