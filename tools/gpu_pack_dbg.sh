#!/bin/bash
# packer phase stamps (LDDL_PACK_DEBUG=1) on the bench workload, per LDS caps
# setting (CAPS_LIST).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-pdbg}
mkdir -p $OUT
for caps in ${CAPS_LIST:-0,0,0}; do
  LDDL_PACK_CAPS=$caps LDDL_PACK_DEBUG=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/b_$caps.log 2>&1 || exit 1
  echo "caps $caps"; grep "pack dbg" $OUT/b_$caps.log
done
