#!/bin/bash
# Row spans with 2 rows per lane (the working tree) against 1 (ab/lib_rs1.so)
# and 4 (ab/lib_rs4.so): kernel trace of a 2-step bench each, alternating;
# then the row-span / materialise tests.
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_rowspan2}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_pack_gpu.py -x -q -m gpu -k "row_spans or materialize" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="bench.py --no-cpu-baseline --parquet-parts 0 --frontend-mb 0 --frontend-c2-mb 0 --legs none --no-sample-check --steps 2 --warmup 1"
for i in 1 2; do
  for L in lddl_amd/liblddl_amd.so ab/lib_rs1.so ab/lib_rs4.so; do
    N=$(basename $L .so)_$i
    LDDL_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$N -o kt --output-format csv -- python -u $B > $OUT/$N.log 2>&1 || { echo "$N failed"; tail -5 $OUT/$N.log; exit 1; }
    f=$(find $OUT/$N -name '*kernel_stats.csv' | head -1)
    echo "$N $(grep -h rowspan_kernel $f | cut -d, -f1-4)" >> $OUT/summary.txt
  done
done
cat $OUT/summary.txt
