#!/bin/bash
# Row spans with XCD-aware blocks (the working tree) against the plain block
# order (ab/lib_rsplain.so, -DLDDL_ROWSPAN_XCD=0): kernel trace of a 2-step
# bench each, twice, alternating; then the row-span tests.
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_rowspan}; mkdir -p $OUT
B="bench.py --no-cpu-baseline --parquet-parts 0 --frontend-mb 0 --frontend-c2-mb 0 --legs none --no-sample-check --steps 2 --warmup 1"
for i in 1 2; do
  for L in lddl_amd/liblddl_amd.so ab/lib_rsplain.so; do
    N=$(basename $L .so)_$i
    LDDL_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$N -o kt --output-format csv -- python -u $B > $OUT/$N.log 2>&1 || { echo "$N failed"; tail -5 $OUT/$N.log; exit 1; }
    f=$(find $OUT/$N -name '*kernel_stats.csv' | head -1)
    echo "$N $(grep -h rowspan_kernel $f | cut -d, -f1-4) $(grep -h '^{' $OUT/$N.log | python3 -c 'import json,sys; print(round(json.load(sys.stdin)["ms_per_step"],2), "ms/step")')"
  done
done | tee $OUT/summary.txt
timeout -k 10 300 python -u -m pytest tests/test_pack_gpu.py -x -q -m gpu -k "row_spans or materialize" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
