#!/bin/bash
# --masking benches (static masking at seq 128 and seq 512) + kernel trace of seq 512.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-mask}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --masking --target-seq-length 128 --no-cpu-baseline > $OUT/bench_m128.log 2>&1; rc=$?; echo "m128 rc=$rc"; tail -1 $OUT/bench_m128.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --masking --target-seq-length 512 --no-cpu-baseline > $OUT/bench_m512.log 2>&1; rc=$?; echo "m512 rc=$rc"; tail -1 $OUT/bench_m512.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --masking > $OUT/kt.log 2>&1; echo "kt rc=$?"
python tools/pmc_summary.py $OUT/kt
