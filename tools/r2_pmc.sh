#!/bin/bash
# PMC passes (one counter group per run, rocprofv3 --pmc) over a command
# given in CMD (default: tokenizer check on a synthetic corpus).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_pmc}; mkdir -p $OUT
export TMPDIR=/tmp
CMD=${CMD:-"python -u tools/tok_check.py ${MB:-256} ${VARIANTS:-5}"}
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
G2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LEVEL_WAVES SQ_ACTIVE_INST_LDS"
G3="FETCH_SIZE"
G4="WRITE_SIZE"
G5="GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL"
i=0
for G in "$G1" "$G2" "$G3" "$G4" "$G5"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $G -d $OUT/p$i -o pmc --output-format csv -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_summary.py $OUT > $OUT/summary.txt; cat $OUT/summary.txt | head -120
