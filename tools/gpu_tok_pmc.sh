#!/bin/bash
# SQ instruction mix of tok4 on tools/tok_check.py (MB, VARIANT) with and
# without the WordPiece ablation (LDDL_TOK_ABLATE=1); one counter group per run.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-tpmc}
mkdir -p $OUT
export TMPDIR=/tmp
G=${G:-SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD}
for abl in 0 1; do
  LDDL_TOK_ABLATE=$abl timeout -s KILL 180 rocprofv3 --pmc $G -d $OUT/p$abl -o pmc --output-format csv -- python tools/tok_check.py ${MB:-1024} ${VARIANT:-4:4} > $OUT/p$abl.log 2>&1 || { echo "pass $abl failed"; exit 1; }
  echo "ablate=$abl $(grep variant $OUT/p$abl.log)"
  python tools/pmc_summary.py $OUT/p$abl | grep -A9 tok4
done
