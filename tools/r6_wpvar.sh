#!/bin/bash
# Round 6: the WordPiece kernel's per-process time at full size -- N separate
# bench processes (headline only), each printing the per-segment kernel
# times of its last step (LDDL_SPLIT_TIMES=1 through Tokenizer.stats()).
#   Usage: N=4 bash tools/r6_wpvar.sh TAG
set -o pipefail
TAG=${1:-r6wpvar}
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out/$TAG
B="bench.py --no-cpu-baseline --no-sample-check --parquet-parts 0 --frontend-mb 0 --frontend-c2-mb 0 --legs none --steps 3 --warmup 1"
for R in $(seq 1 ${N:-4}); do
  timeout -k 10 400 python -u $B > gpurun_out/$TAG/run$R.log 2>&1 || { tail -20 gpurun_out/$TAG/run$R.log; exit 1; }
  grep '^{' gpurun_out/$TAG/run$R.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('run $R', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['tokenize_kernels_ms'].items()})"
done
