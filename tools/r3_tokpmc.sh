#!/bin/bash
# Tokenizer kernels' PMC passes on MB of synthetic Wikipedia-style text (one
# counter group per rocprofv3 run, each bounded), then a summary.
#   TAG=r3_tokpmc MB=1024 tools/r3_tokpmc.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r3_tokpmc}
mkdir -p $OUT
export TMPDIR=/tmp NOCHECK=1
B="tools/tok_check.py ${MB:-1024} 5"
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
G2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"
G3="GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_UNALIGNED_STALL"
G4="FETCH_SIZE"
G5="WRITE_SIZE"
i=0
for G in "$G1" "$G2" "$G3" "$G4" "$G5"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $G -d $OUT/p$i -o pmc --output-format csv -- python -u $B > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt; grep -A30 'scan_kernel\|wp_kernel\|expand_kernel' $OUT/pmc_summary.txt | head -100
