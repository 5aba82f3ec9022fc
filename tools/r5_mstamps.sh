#!/bin/bash
# Masked packer phase stamps (LDDL_PACK_DEBUG=1: the stamped kernel build,
# s_memtime ticks summed over waves) of a 1-step --masking bench at seq 512
# and seq 128, for each library in LIBS (default: the working tree's).
#   TAG=r5_mst LIBS="lddl_amd/liblddl_amd.so ab/lib_x.so" bash tools/r5_mstamps.sh
set -o pipefail
O=gpurun_out/${TAG:-r5_mst}
mkdir -p $O
export TMPDIR=/tmp
B="bench.py --masking --no-cpu-baseline --parquet-parts 0 --frontend-mb 0 --frontend-c2-mb 0 --legs none --no-sample-check --steps 1 --warmup 1"
for L in ${LIBS:-lddl_amd/liblddl_amd.so}; do
  N=$(basename $L .so)
  for SEQ in 512 128; do
    LDDL_LIB=$PWD/$L LDDL_PACK_DEBUG=1 timeout -k 10 300 python -u $B --target-seq-length $SEQ > $O/${N}_$SEQ.log 2>&1 || { tail -5 $O/${N}_$SEQ.log; exit 1; }
    LDDL_LIB=$PWD/$L timeout -k 10 300 python -u $B --target-seq-length $SEQ --steps 3 > $O/${N}_${SEQ}_t.log 2>&1 || { tail -5 $O/${N}_${SEQ}_t.log; exit 1; }
    echo "$N seq $SEQ: $(grep -h 'lddl pack dbg' $O/${N}_$SEQ.log | tail -1)"
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/${N}_${SEQ}_t.log') if l.startswith('{')][-1]); print('  ms/step', round(d['ms_per_step'],1))"
  done
done
