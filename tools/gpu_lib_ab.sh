#!/bin/bash
# A/B of the whole bench step: in-tree library (A) vs lddl_amd/liblddl_amd_b.so
# (B), each under a kernel trace; prints per-kernel averages.  BENCH_ARGS adds
# bench flags.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-libab}
mkdir -p $OUT
export TMPDIR=/tmp
for v in a b; do
  if [ $v = b ]; then export LDDL_LIB=$GRAFT_REPO_ROOT/lddl_amd/liblddl_amd_b.so; fi
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt_$v -o kt --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --parquet-parts 0 ${BENCH_ARGS} > $OUT/kt_$v.log 2>&1 || { echo "$v failed"; exit 1; }
  echo "== $v: $(tail -1 $OUT/kt_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  python tools/pmc_summary.py $OUT/kt_$v | head -5
done
