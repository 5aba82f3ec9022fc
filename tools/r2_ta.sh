#!/bin/bash
# TA / TCP (vector memory front end) counters on the tokenizer kernels
# (tools/tok_check.py, 512 MB): one rocprofv3 --pmc pass per group.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_ta}; mkdir -p $OUT
export TMPDIR=/tmp
i=0
for G in "TA_BUSY_avr TA_TOTAL_WAVEFRONTS_sum GRBM_GUI_ACTIVE" \
         "TCP_TCP_TA_ADDR_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
         "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
         "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $G -d $OUT/p$i -o pmc --output-format csv -- python -u tools/tok_check.py ${MB:-512} 5 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_summary.py $OUT > $OUT/summary.txt; grep -A14 "scan_kernel\|wp_kernel\|expand_kernel" $OUT/summary.txt | head -60
