#!/bin/bash
# materialize bring-up: pack GPU tests, then kernel trace of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-mat}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_pack_gpu.py} > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/kt.log 2>&1; echo "kt rc=$?"
tail -1 $OUT/kt.log | cut -c1-300
python tools/pmc_summary.py $OUT/kt
