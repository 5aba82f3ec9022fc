#!/bin/bash
# masking packer: GPU parity tests, then --masking bench per LDDL_MASK_DIAG variant
# (0: batched shuffle draws + 16-B swap reads; 2: u16 reads; 4: readlane; 1: sequential draws).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-mask_ab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pack_gpu.py tests/test_preprocess.py tests/test_writer_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
for v in ${VARIANTS:-0 2 4 1}; do
  LDDL_MASK_DIAG=$v timeout -k 10 600 python bench.py --masking --no-cpu-baseline --steps 2 > $OUT/bench_m512_v$v.log 2>&1; rc=$?
  echo "variant $v rc=$rc"; tail -1 $OUT/bench_m512_v$v.log | cut -c1-330
  [ $rc -ne 0 ] && exit $rc
done
[ -n "$NO_KT" ] && exit 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --masking > $OUT/kt.log 2>&1; echo "kt rc=$?"
python tools/pmc_summary.py $OUT/kt
