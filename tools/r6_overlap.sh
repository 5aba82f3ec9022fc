#!/bin/bash
# Round 6: the bench step with and without the two-stream step overlap,
# alternating, headline only (no CPU baseline / CLI legs / other legs); the
# full-size partition check stays on.   Usage: bash tools/r6_overlap.sh TAG
set -o pipefail
TAG=${1:-r6ov}
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out/$TAG
B="bench.py --cpu-seconds 2 --parquet-parts 0 --frontend-mb 0 --frontend-c2-mb 0 --legs none --steps ${STEPS:-5} --warmup 1"
for R in 1 2; do
  for M in overlap no-overlap; do
    timeout -k 10 400 python -u $B --$M > gpurun_out/$TAG/$M.$R.log 2>&1 || { tail -20 gpurun_out/$TAG/$M.$R.log; exit 1; }
    grep '^{' gpurun_out/$TAG/$M.$R.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$M', d['ms_per_step'], d['value']/1e9, d['config'].get('step_overlap'), d.get('cpu_baseline', {}).get('sample_check'))"
  done
done
