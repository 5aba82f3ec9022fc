#!/bin/bash
# Tokenizer v4 bring-up session: parity + timing of the variants, phase
# stamps, kernel trace, then (TESTS=...) GPU tests.  Every GPU step bounded;
# stops at a crash.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-tok4}
mkdir -p $OUT
export TMPDIR=/tmp
ok() { local rc=$1; [ $rc -lt 124 ] || { echo "step failed rc=$rc"; exit $rc; }; }
timeout -k 10 300 python tools/tok_check.py ${MB:-64} ${VARIANTS:-3 4:0 4:1 4:2 4:3} > $OUT/tok_check.log 2>&1; ok $?
grep variant $OUT/tok_check.log
LDDL_TOK_DEBUG=1 timeout -k 10 300 python tools/tok_check.py ${MB:-64} ${DBG_VARIANTS:-4:0 4:1} > $OUT/tok_dbg.log 2>&1; ok $?
grep "tok4 dbg" $OUT/tok_dbg.log | awk 'NR%4==0'
if [ -n "$TRACE" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python tools/tok_check.py ${MB:-64} $TRACE > $OUT/kt.log 2>&1; ok $?
  cat $(find $OUT/kt -name '*kernel_stats.csv') | cut -d, -f1-4 | head -8
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $OUT/pytest.log 2>&1
  echo "pytest rc=$?"; tail -5 $OUT/pytest.log
fi
