#!/bin/bash
# Kernel-trace A/B of library builds on the default bench (2 steps each).
#   LIBS="ab/lib_a.so" BENCH_ARGS="--masking" tools/r2_trace_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_trace_ab}; mkdir -p $OUT
export TMPDIR=/tmp
for L in lddl_amd/liblddl_amd.so ${LIBS}; do
  N=$(basename $L .so)
  LDDL_LIB=$PWD/$L timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/$N -o kt --output-format csv -- python -u bench.py --no-cpu-baseline --parquet-parts 0 --steps 2 --warmup 1 ${BENCH_ARGS} > $OUT/$N.log 2>&1 || { tail -20 $OUT/$N.log; exit 1; }
  echo "== $N"
  grep -h '"metric"' $OUT/$N.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms_per_step %.2f' % d['ms_per_step'], d.get('tokenize_kernels_ms'))"
  f=$(find $OUT/$N -name '*kernel_stats.csv' | head -1)
  python - $f <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print('  %-50s %4s %9.3f ms/call %9.2f total' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e6, float(r['TotalDurationNs'])/1e6))
PY
done
