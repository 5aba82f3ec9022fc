#!/bin/bash
# Diagnostics: FETCH calibration (tools/fetch_calib) + packer phase stamps on
# the bench workload (LDDL_PACK_DEBUG=1) + tokenizer phase stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_probe}; mkdir -p $OUT
export TMPDIR=/tmp
TAG=$(basename $OUT)/calib timeout -k 10 300 tools/gpu_calib.sh > $OUT/calib.log 2>&1 || { echo "calib failed"; tail $OUT/calib.log; exit 1; }
cat $OUT/calib.log
LDDL_PACK_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --parquet-parts 0 ${BENCH_ARGS} > $OUT/packdbg.log 2>&1 || { echo "packdbg failed"; tail $OUT/packdbg.log; exit 1; }
grep "pack dbg" $OUT/packdbg.log
