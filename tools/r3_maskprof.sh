#!/bin/bash
# Masked packer (BERT seq 512, --masking): phase stamps (LDDL_PACK_DEBUG=1),
# a kernel trace and two PMC passes of a 4 GB bench step.   TAG=x [LIBS="ab/lib_a.so ..."] tools/r3_maskprof.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-maskprof}; mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --masking --corpus-gb ${GB:-4} --no-cpu-baseline --frontend-mb 0 --parquet-parts 0 --no-sample-check"
for L in lddl_amd/liblddl_amd.so ${LIBS}; do
  N=$(basename $L .so)
  echo "== $N"
  if [ -z "$SKIP_DBG" ]; then
    LDDL_LIB=$PWD/$L LDDL_PACK_DEBUG=1 timeout -k 10 300 python -u $B --steps 1 --warmup 0 > $OUT/dbg_$N.log 2>&1 || { echo "dbg $N failed"; tail $OUT/dbg_$N.log; exit 1; }
    grep "pack dbg" $OUT/dbg_$N.log | tail -1
  fi
  LDDL_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_$N -o kt --output-format csv -- python -u $B --steps ${KT_STEPS:-2} --warmup 1 > $OUT/kt_$N.log 2>&1 || { echo "kt $N failed"; tail $OUT/kt_$N.log; exit 1; }
  f=$(find $OUT/kt_$N -name '*kernel_stats.csv' | head -1); grep pack_bert $f | cut -d, -f1-4
done
[ -n "$SKIP_PMC" ] && exit 0
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
G2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"
G3="GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA"
i=0
for G in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $G -d $OUT/p$i -o pmc --output-format csv -- python -u $B --steps 1 --warmup 0 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt; grep -A24 'pack_bert_wave_kernel<1' $OUT/pmc_summary.txt | head -26
