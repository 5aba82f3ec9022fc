#!/bin/bash
# Tokenizer A/B of library builds (ab/lib_*.so from tools/ab_build.py, and the
# main build) on the same synthetic corpus: parity + per-kernel times.
#   LIBS="ab/lib_a.so ab/lib_b.so" MB=512 tools/r2_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_ab}; mkdir -p $OUT
for L in lddl_amd/liblddl_amd.so ${LIBS:-ab/lib_*.so}; do
  N=$(basename $L .so)
  LDDL_LIB=$PWD/$L timeout -k 10 300 env $TOKENV python -u tools/tok_check.py ${MB:-512} 5 > $OUT/$N.log 2>&1 || { echo "$N failed"; tail $OUT/$N.log; exit 1; }
  echo "== $N"; grep -v "amdgpu.ids\|^gen" $OUT/$N.log
done
