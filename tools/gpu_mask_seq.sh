#!/bin/bash
# masking packer parity + --masking benches at seq 128 and 512 + kernel trace of seq 512.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-mask_seq}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pack_gpu.py tests/test_preprocess.py tests/test_writer_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
for sl in 128 512; do
  timeout -k 10 600 python bench.py --masking --target-seq-length $sl --no-cpu-baseline --steps 2 > $OUT/bench_m$sl.log 2>&1; rc=$?
  echo "seq $sl rc=$rc"; tail -1 $OUT/bench_m$sl.log | cut -c1-330
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --masking > $OUT/kt.log 2>&1; echo "kt rc=$?"
python tools/pmc_summary.py $OUT/kt
