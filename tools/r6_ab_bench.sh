#!/bin/bash
# Round 6: headline bench step (no CPU baseline / CLI legs / other legs, no
# partition check) for the working tree's library and each LIBS entry, in
# forward then reverse order.   Usage: [LIBS=ab/lib_x.so] [ARGS=...] bash tools/r6_ab_bench.sh TAG
set -o pipefail
TAG=${1:-r6ab}
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out/$TAG
B="bench.py --no-cpu-baseline --no-sample-check --parquet-parts 0 --frontend-mb 0 --frontend-c2-mb 0 --legs none --steps ${STEPS:-3} --warmup 1 $ARGS"
ORDER="lddl_amd/liblddl_amd.so ${LIBS}"
REV=""; for L in $ORDER; do REV="$L $REV"; done
for L in $ORDER $REV; do
  N=$(basename $L .so)
  LDDL_LIB=$PWD/$L timeout -k 10 400 python -u $B >> gpurun_out/$TAG/$N.log 2>&1 || { tail -20 gpurun_out/$TAG/$N.log; exit 1; }
  grep '^{' gpurun_out/$TAG/$N.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$N', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['tokenize_kernels_ms'].items()}, round(d['roofline']['avg_launch_ms'],3))"
done
