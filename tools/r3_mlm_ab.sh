#!/bin/bash
# masked_lm_kernel A/B: the pack / writer GPU tests on LIB, then a kernel trace
# of a 20 GB masked bench step with LIB and with REF.   LIB=ab/lib_x.so REF=ab/lib_head.so TAG=x tools/r3_mlm_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-mlm_ab}; mkdir -p $OUT
export TMPDIR=/tmp
LDDL_LIB=$PWD/$LIB timeout -k 10 400 python -u -m pytest tests/test_pack_gpu.py tests/test_writer_gpu.py tests/test_preprocess.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; grep -E "Error|FAILED|assert" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="bench.py --masking --no-cpu-baseline --frontend-mb 0 --parquet-parts 0 --no-sample-check"
for L in $LIB $REF; do
  N=$(basename $L .so)
  LDDL_LIB=$PWD/$L timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt_$N -o kt --output-format csv -- python -u $B --steps 1 --warmup 1 > $OUT/kt_$N.log 2>&1 || { echo "kt $N failed"; tail $OUT/kt_$N.log; exit 1; }
  f=$(find $OUT/kt_$N -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats_$N.csv
  echo "== $N $(tail -1 $OUT/kt_$N.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],1), "ms/step")')"
  grep -E "masked_lm|pack_bert|materialize" $f | cut -d, -f1-4
done
