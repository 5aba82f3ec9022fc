#!/bin/bash
# Round 5: PMC passes of the tokenizer (tools/tok_check.py, variant 6 or
# $VARIANT) on MB of synthetic text; one counter group per bounded pass.
set -o pipefail
TAG=${1:-r5tokpmc}; MB=${2:-256}
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && OUT=gpurun_out/$TAG && mkdir -p $OUT
i=0
while read -r G; do
  [ -z "$G" ] && continue
  i=$((i+1))
  NOCHECK=1 timeout -s KILL 240 rocprofv3 --pmc $G -d $OUT/pmc_$i -o pmc --output-format csv -- python tools/tok_check.py $MB ${VARIANT:-6} > $OUT/pmc_$i.log 2>&1 || { echo "pass $i ($G) failed"; tail -5 $OUT/pmc_$i.log; exit 1; }
  python tools/pmc_summary.py $OUT/pmc_$i > $OUT/pmc_$i.txt
done <<< "${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES
SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE TA_BUSY_avr TA_TOTAL_WAVEFRONTS_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_ADDR_STALL_CYCLES_sum
TCC_HIT_sum TCC_MISS_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum
FETCH_SIZE
WRITE_SIZE}"
cat $OUT/pmc_*.txt > $OUT/summary.txt
