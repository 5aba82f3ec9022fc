#!/bin/bash
# Round 6: the -m gpu suite (skips named) and smoke() on the working tree.
set -o pipefail
TAG=${1:-r6t}
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -x -q -rs -m gpu --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
