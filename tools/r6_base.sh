set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r6base
timeout -k 10 300 python -u tools/tok_check.py 1024 5 > gpurun_out/r6base/tok.txt 2>&1 || exit $?
LDDL_TOK_DEBUG=1 NOCHECK=1 timeout -k 10 300 python -u tools/tok_check.py 1024 5 > gpurun_out/r6base/stamps.txt 2>&1 || exit $?
