#!/bin/bash
# Round 5: lane tokenizer (tok6) on the GPU -- parity + timing (+ phase
# stamps with STAMPS=1) against tok5 in one call; pytest of the tokenizer
# suite unless NOTEST=1.   Usage (GPU box): bash tools/r5_tok.sh TAG [MB]
set -o pipefail
TAG=${1:-r5tok}; MB=${2:-1024}
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out/$TAG
LDDL_LANE_STATS=1 timeout -k 10 300 python -u tools/tok_check.py $MB 6 5 > gpurun_out/$TAG/tok_check.txt 2>&1 || exit $?
if [ -n "$STAMPS" ]; then
  LDDL_LANE_STATS=2 NOCHECK=1 timeout -k 10 300 python -u tools/tok_check.py $MB 6 > gpurun_out/$TAG/tok_stamps.txt 2>&1 || exit $?
fi
for L in ${LIBS}; do
  N=$(basename $L .so)
  LDDL_LIB=$PWD/$L LDDL_LANE_STATS=1 timeout -k 10 300 python -u tools/tok_check.py $MB 6 > gpurun_out/$TAG/$N.txt 2>&1 || exit $?
done
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tokenize_gpu.py \
    > gpurun_out/$TAG/pytest_tok.txt 2>&1
fi
