#!/bin/bash
# Full GPU session: tests, smoke, default bench, kernel trace of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-full}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $OUT/smoke.log
timeout -k 10 900 python bench.py ${BENCH_ARGS} > $OUT/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/kt.log 2>&1; echo "kt rc=$?"
python tools/pmc_summary.py $OUT/kt
