#!/bin/bash
# Tokenizer A/B on a synthetic corpus (tools/tok_check.py): parity on the
# first MBs + per-kernel times.  MB / VARIANTS / TOKENV from the env.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_tok}; mkdir -p $OUT
timeout -k 10 300 env $TOKENV python -u tools/tok_check.py ${MB:-1024} ${VARIANTS:-5} > $OUT/check.log 2>&1; rc=$?
grep -v amdgpu.ids $OUT/check.log; exit $rc
