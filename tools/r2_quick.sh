#!/bin/bash
# Quick check of the current tree: the GPU tests (optionally filtered by
# K="expr"), then a kernel trace of a 2-step bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_quick}; mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu ${K:+-k "$K"} --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python -u bench.py --no-cpu-baseline --parquet-parts 0 --steps 2 --warmup 1 ${BENCH_ARGS} > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
tail -1 $OUT/kt.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms_per_step', d['ms_per_step'], 'value', d['value'], d.get('tokenize_kernels_ms'))"
f=$(find $OUT/kt -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats.csv
python - $f <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:9]:
    print('%-60s %6s %10.3f ms/call %9.2f ms total' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e6, float(r['TotalDurationNs'])/1e6))
PY
