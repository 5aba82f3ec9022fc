#!/bin/bash
# CodeBERT bench (configs[2] on one GPU) + its kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-code}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --corpus code > $OUT/bench_code.log 2>&1; rc=$?; echo "bench code rc=$rc"; tail -1 $OUT/bench_code.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt_code -o kt --output-format csv -- python bench.py --corpus code --steps 2 --warmup 1 --no-cpu-baseline --parquet-parts 0 > $OUT/kt_code.log 2>&1; echo "kt rc=$?"
python tools/pmc_summary.py $OUT/kt_code
