#!/bin/bash
# expand_kernel EXP_K: kernel traces of a 2-step bench for the tree's library
# and ab/lib_ek.so, alternating, twice each (expand per-launch average).
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/ek
B="bench.py --no-cpu-baseline --no-sample-check --parquet-parts 0 --frontend-mb 0 --frontend-c2-mb 0 --legs none --steps 2 --warmup 1"
k=0
for L in lddl_amd/liblddl_amd.so ab/lib_ek.so ab/lib_ek.so lddl_amd/liblddl_amd.so; do
  k=$((k+1)); N=$(basename $L .so)_$k
  LDDL_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ek/$N -o kt --output-format csv -- python -u $B > gpurun_out/ek/$N.log 2>&1 || { tail -5 gpurun_out/ek/$N.log; exit 1; }
  f=$(find gpurun_out/ek/$N -name '*kernel_stats.csv' | head -1); cp $f gpurun_out/ek/${N}_stats.csv
  echo $N $(grep -h 'expand_kernel' $f | awk -F'",' '{print $2}' | cut -d, -f1-3)
done
