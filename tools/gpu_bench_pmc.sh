#!/bin/bash
# PMC passes over a 1-step bench (one counter group per run, PMC_GROUPS one
# group a line; default the HBM traffic pair FETCH_SIZE / WRITE_SIZE);
# per-kernel means under gpurun_out/$TAG/.  Every pass bounded; stops at the
# first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-bpmc}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
while read -r G; do
  [ -z "$G" ] && continue
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $G -d $OUT/pmc_$i -o pmc --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} > $OUT/pmc_$i.log 2>&1 || { echo "pass $i ($G) failed"; exit 1; }
  python tools/pmc_summary.py $OUT/pmc_$i > $OUT/pmc_$i.txt
  cat $OUT/pmc_$i.txt
done <<< "${PMC_GROUPS:-FETCH_SIZE
WRITE_SIZE}"
