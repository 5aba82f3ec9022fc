#!/bin/bash
# Kernel trace of the tokenizer variants on a synthetic corpus (tok_check).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_tokprof}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python -u tools/tok_check.py ${MB:-256} ${VARIANTS:-5} > $OUT/kt.log 2>&1; rc=$?
grep -h variant $OUT/kt.log
f=$(find $OUT/kt -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 $f | head -14
exit $rc
