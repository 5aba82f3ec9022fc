#!/bin/bash
# Tokenizer instruction mix (one --pmc pass) + timing on the mixed and the
# ASCII-only synthetic corpus.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_tokpmc}; mkdir -p $OUT
export TMPDIR=/tmp
G="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for A in 0 1; do
  ASCII=$A timeout -k 10 200 python -u tools/tok_check.py ${MB:-256} 5 > $OUT/t$A.log 2>&1 || { echo "tok_check failed"; tail $OUT/t$A.log; exit 1; }
  grep -v amdgpu.ids $OUT/t$A.log | tail -2
  ASCII=$A timeout -s KILL 200 rocprofv3 --pmc $G -d $OUT/p$A -o pmc --output-format csv -- python -u tools/tok_check.py ${MB:-256} 5 > $OUT/p$A.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/p$A.log; exit 1; }
  python tools/pmc_summary.py $OUT/p$A | grep -A9 "scan_kernel\|wp_kernel\|expand_kernel"
done
