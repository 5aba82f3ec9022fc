#!/bin/bash
# materialize phase split: kernel trace of a 1-step bench with and without the
# edge-chunk drain (LDDL_MAT_ABLATE=1, wrong output: diagnostics only)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-matabl}
mkdir -p $OUT
export TMPDIR=/tmp
for a in 0 1; do
  LDDL_MAT_ABLATE=$a timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/k$a -o kt --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/k$a.log 2>&1 || { echo "run $a failed"; exit 1; }
  echo "ablate=$a"; python tools/pmc_summary.py $OUT/k$a | grep -E "materialize|compact"
done
