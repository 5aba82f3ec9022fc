#!/bin/bash
# GPU-box session: tests, smoke, bench, rocprof kernel trace (each step bounded).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> $OUT/status
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; echo "smoke rc=$?" >> $OUT/status
tail -2 $OUT/smoke.log
timeout -k 10 900 python bench.py ${BENCH_ARGS} > $OUT/bench.log 2>&1; echo "bench rc=$?" >> $OUT/status
tail -2 $OUT/bench.log
cat $OUT/status
