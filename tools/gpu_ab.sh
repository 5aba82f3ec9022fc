#!/bin/bash
# A/B timing of the tokenizer: the in-tree library (A) against
# lddl_amd/liblddl_amd_b.so (B, e.g. built from HEAD), interleaved A B A B.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python tools/tok_check.py ${MB:-2048} ${VARIANTS:-4:4} > $OUT/a$r.log 2>&1 || { echo "A failed"; exit 1; }
  echo "A: $(grep variant $OUT/a$r.log)"
  LDDL_LIB=$GRAFT_REPO_ROOT/lddl_amd/liblddl_amd_b.so timeout -k 10 300 python tools/tok_check.py ${MB:-2048} ${VARIANTS:-4:4} > $OUT/b$r.log 2>&1 || { echo "B failed"; exit 1; }
  echo "B: $(grep variant $OUT/b$r.log)"
done
