#!/bin/bash
# count_kernel sentences per thread: GPU tokenizer tests on the tree's library,
# then a kernel trace of a 2-step bench for it and ab/lib_cnt1.so.
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/cnt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tokenize_gpu.py > gpurun_out/cnt/pt.log 2>&1 || { tail -20 gpurun_out/cnt/pt.log; exit 1; }
tail -1 gpurun_out/cnt/pt.log
B="bench.py --no-cpu-baseline --no-sample-check --parquet-parts 0 --frontend-mb 0 --frontend-c2-mb 0 --legs none --steps 2 --warmup 1"
for L in lddl_amd/liblddl_amd.so ab/lib_cnt1.so; do
  N=$(basename $L .so)
  LDDL_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cnt/$N -o kt --output-format csv -- python -u $B > gpurun_out/cnt/$N.log 2>&1 || { tail -5 gpurun_out/cnt/$N.log; exit 1; }
  f=$(find gpurun_out/cnt/$N -name '*kernel_stats.csv' | head -1); cp $f gpurun_out/cnt/${N}_stats.csv
  echo $N $(grep -h 'count_kernel' $f | cut -d, -f2-4) $(grep '^{' gpurun_out/cnt/$N.log | python3 -c "import json,sys; print(round(json.load(sys.stdin)['ms_per_step'],2))")
done
