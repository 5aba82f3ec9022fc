#!/bin/bash
# masked packer phase stamps (LDDL_PACK_DEBUG=1) at seq 128 and 512.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-mask_dbg}
mkdir -p $OUT
for sl in 128 512; do
  LDDL_PACK_DEBUG=1 timeout -k 10 600 python bench.py --masking --target-seq-length $sl --no-cpu-baseline --steps 1 --warmup 1 > $OUT/dbg_m$sl.log 2>&1; rc=$?
  echo "seq $sl rc=$rc"; grep "pack dbg" $OUT/dbg_m$sl.log | tail -1
  [ $rc -ne 0 ] && exit $rc
done
exit 0
