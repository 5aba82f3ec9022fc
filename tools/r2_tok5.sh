#!/bin/bash
# v5 split tokenizer bring-up: parity + timing vs tok4, then the tokenizer GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_tok5}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/tok_check.py ${MB:-64} ${VARIANTS:-4:4 5} > $OUT/check.log 2>&1; rc=$?
grep -h "variant\|differ\|Error\|error" $OUT/check.log | head -20
[ $rc -ne 0 ] && { tail -20 $OUT/check.log; exit $rc; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tokenize_gpu.py -k "${PYK:-tokenize}" > $OUT/pytest.log 2>&1; rc=$?
tail -15 $OUT/pytest.log
exit $rc
