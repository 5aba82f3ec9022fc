#!/bin/bash
# Round 6: tokenizer A/B on the GPU box -- tools/tok_check.py (parity on a
# 27 908-sentence sample + timing, min of 3) for the working tree's library
# and every LIBS entry (ab/lib_*.so), phase stamps with STAMPS=1, the
# tokenizer test suite unless NOTEST=1.   Usage: bash tools/r6_tok.sh TAG [MB]
set -o pipefail
TAG=${1:-r6tok}; MB=${2:-1024}
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out/$TAG
# (each library twice, the second time in reverse order: the first run of a
# call measured ~1 % slower with identical code, profiles/r6/h1_*; compare
# the min of each library's lines)
ORDER="lddl_amd/liblddl_amd.so ${LIBS}"
REV=""; for L in $ORDER; do REV="$L $REV"; done
[ -n "${LIBS}" ] && ORDER="$ORDER $REV"
for L in $ORDER; do
  N=$(basename $L .so)
  LDDL_LIB=$PWD/$L timeout -k 10 300 python -u tools/tok_check.py $MB 5 >> gpurun_out/$TAG/$N.txt 2>&1 || { tail -5 gpurun_out/$TAG/$N.txt; exit 1; }
done
if [ -n "$STAMPS" ]; then
  LDDL_TOK_DEBUG=1 NOCHECK=1 timeout -k 10 300 python -u tools/tok_check.py $MB 5 > gpurun_out/$TAG/stamps.txt 2>&1 || exit $?
fi
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest -x -v -rs --timeout 300 --timeout-method thread tests/test_tokenize_gpu.py \
    > gpurun_out/$TAG/pytest_tok.txt 2>&1
fi
