#!/bin/bash
# PC sampling (rocprofv3 beta, host_trap) of a small tokenizer or pack run.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_pcs}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/list.log 2>&1; grep -i -B2 -A12 "pc_sampl\|PC sampling" $OUT/list.log | head -60
CMD=${CMD:-"python -u tools/tok_check.py 64 5"}
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${METHOD:-host_trap} --pc-sampling-unit ${UNIT:-time} --pc-sampling-interval ${IVL:-1} -d $OUT/pcs -o pcs --output-format csv -- $CMD > $OUT/pcs.log 2>&1; rc=$?
tail -5 $OUT/pcs.log; find $OUT/pcs -type f | head; exit $rc
