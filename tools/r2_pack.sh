#!/bin/bash
# Packer A/B: GPU pack/writer parity tests, phase stamps, a short bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_pack}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_pack_gpu.py tests/test_writer_gpu.py} -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
LDDL_PACK_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --parquet-parts 0 ${BENCH_ARGS} > $OUT/packdbg.log 2>&1 || { echo "packdbg failed"; tail $OUT/packdbg.log; exit 1; }
grep "pack dbg" $OUT/packdbg.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --parquet-parts 0 ${BENCH_ARGS} > $OUT/kt.log 2>&1 || { echo "kt failed"; tail $OUT/kt.log; exit 1; }
tail -1 $OUT/kt.log | cut -c1-400
f=$(find $OUT/kt -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 $f | head -12
