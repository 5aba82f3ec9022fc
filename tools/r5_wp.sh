#!/bin/bash
# Round 5: split tokenizer with the trie-walk WordPiece kernel (default)
# against the Bloom-scan one (LDDL_WP_ALGO=bloom) in one call, then the
# tokenizer test suite.  Usage (GPU box): bash tools/r5_wp.sh TAG [MB]
set -o pipefail
TAG=${1:-r5wp}; MB=${2:-1024}
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u tools/tok_check.py $MB 5 > gpurun_out/$TAG/tok_trie.txt 2>&1 || exit $?
LDDL_WP_ALGO=bloom timeout -k 10 300 python -u tools/tok_check.py $MB 5 > gpurun_out/$TAG/tok_bloom.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/tok_check.py $MB 5 > gpurun_out/$TAG/tok_trie2.txt 2>&1 || exit $?
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tokenize_gpu.py \
    > gpurun_out/$TAG/pytest_tok.txt 2>&1
fi
