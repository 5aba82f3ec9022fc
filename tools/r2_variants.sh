#!/bin/bash
# The workload variants of bench.py (static masking seq 512, CodeBERT,
# Wikipedia+Books), one bench line each, plus a kernel trace of the masked
# bench.  Each GPU step bounded; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_variants}; mkdir -p $OUT
export TMPDIR=/tmp
for v in "default:" "mask512:--masking" "code:--corpus code" "wikibooks:--corpus wikibooks"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 900 python -u bench.py $a > $OUT/bench_$n.log 2>&1 || { echo "$n failed"; tail -20 $OUT/bench_$n.log; exit 1; }
  grep -h '"metric"' $OUT/bench_$n.log | tail -1 > $OUT/bench_$n.json
  python -c "import json; d=json.load(open('$OUT/bench_$n.json')); print('$n', round(d['value']/1e9,3), 'G tok/s', round(d['ms_per_step'],1), 'ms', d['cpu_baseline'].get('sample_check'))"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/mkt -o kt --output-format csv -- python -u bench.py --masking --no-cpu-baseline --parquet-parts 0 --steps 2 --warmup 1 > $OUT/mkt.log 2>&1 || { tail $OUT/mkt.log; exit 1; }
f=$(find $OUT/mkt -name '*kernel_stats.csv' | head -1); cp $f $OUT/mask_kernel_stats.csv; cut -d, -f1-4 $f | head -8
