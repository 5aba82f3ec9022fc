#!/bin/bash
# Masked step (seq 512 by default) kernel trace and counter passes: which
# kernels the masked bench step spends its time in.   Usage: [SEQ=512] bash tools/r6_mask_prof.sh TAG
set -o pipefail
TAG=${1:-r6mask}
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && OUT=gpurun_out/$TAG && mkdir -p $OUT
B="bench.py --masking --target-seq-length ${SEQ:-512} --no-cpu-baseline --no-sample-check --parquet-parts 0 --frontend-mb 0 --frontend-c2-mb 0 --legs none"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python -u $B --steps 2 --warmup 1 > $OUT/kt.log 2>&1 || { echo "kernel trace failed"; tail -20 $OUT/kt.log; exit 1; }
f=$(find $OUT/kt -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats.csv
python3 -c "
import csv
for r in list(csv.reader(open('$OUT/kernel_stats.csv')))[1:9]: print(r[0][:70], r[1], round(float(r[3])/1e6,3), 'ms avg')"
[ -n "$SKIP_PMC" ] && exit 0
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
G2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"
G3="FETCH_SIZE"
G4="WRITE_SIZE"
i=0
for G in "$G1" "$G2" "$G3" "$G4"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $G -d $OUT/p$i -o pmc --output-format csv -- python -u $B --steps 1 --warmup 0 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt; grep -A16 'masked_lm_spans' $OUT/pmc_summary.txt | head -18
