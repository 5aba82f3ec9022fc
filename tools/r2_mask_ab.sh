#!/bin/bash
# Masked packer A/B: the masked GPU tests on the main build, then the
# --masking bench (and the packer's phase stamps) for each library build.
#   LIBS="ab/lib_a.so ab/lib_b.so" tools/r2_mask_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_mask_ab}; mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_pack_gpu.py -x -q -k "mask" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for L in lddl_amd/liblddl_amd.so ${LIBS}; do
  N=$(basename $L .so)
  LDDL_LIB=$PWD/$L LDDL_PACK_DEBUG=1 timeout -k 10 600 python -u bench.py --masking --no-cpu-baseline --parquet-parts 0 --steps 2 --warmup 1 ${BENCH_ARGS} > $OUT/$N.log 2>&1 || { echo "$N failed"; tail $OUT/$N.log; exit 1; }
  echo "== $N"; grep "pack dbg" $OUT/$N.log | tail -1
  tail -1 $OUT/$N.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms_per_step', d['ms_per_step'], 'value', d['value'])"
done
