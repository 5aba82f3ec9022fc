#!/bin/bash
# PMC passes (one counter group per run) over tools/tok_check.py for one
# tokenizer variant; summaries under gpurun_out/$TAG/pmc_*.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
export TMPDIR=/tmp
V=${V:-4:2}
i=0
while read -r G; do
  [ -z "$G" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G -d $OUT/pmc_$i -o pmc --output-format csv -- python tools/tok_check.py ${MB:-64} $V > $OUT/pmc_$i.log 2>&1 || { echo "pass $i ($G) failed"; exit 1; }
  python tools/pmc_summary.py $OUT/pmc_$i tok4_kernel 2>/dev/null || find $OUT/pmc_$i -name '*counter_collection.csv' | head -1
done <<< "${PMC_GROUPS:-FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_LDS}"
