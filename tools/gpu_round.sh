#!/bin/bash
# Round-end style session: tests, smoke, bench (with cpu baseline), rocprof
# kernel trace + PMC passes of the bench.  Each GPU step bounded; stops at
# the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-round}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 900 python bench.py ${BENCH_ARGS} > $OUT/bench.log 2>&1 && echo "bench ok" && tail -1 $OUT/bench.log &&
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline ${PROF_ARGS}" &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python $B > $OUT/kt.log 2>&1 && echo "kt ok" &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o pmc --output-format csv -- python $B > $OUT/pmc_fetch.log 2>&1 && echo "fetch ok" &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o pmc --output-format csv -- python $B > $OUT/pmc_write.log 2>&1 && echo "write ok"
tail -3 $OUT/pytest_gpu.log
