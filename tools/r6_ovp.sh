#!/bin/bash
# Round 6: the bench step with the two-stream overlap, the pack stream at the
# higher priority (1) or not (0), and without the overlap, alternating.
#   Usage: bash tools/r6_ovp.sh TAG
set -o pipefail
TAG=${1:-r6ovp}
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out/$TAG
B="bench.py --no-cpu-baseline --parquet-parts 0 --frontend-mb 0 --frontend-c2-mb 0 --legs none --steps ${STEPS:-5} --warmup 1"
for R in 1 2; do
  for M in "--overlap --overlap-priority 1" "--overlap --overlap-priority 0" "--no-overlap"; do
    N=$(echo $M | tr -d ' -')
    timeout -k 10 400 python -u $B $M > gpurun_out/$TAG/$N.$R.log 2>&1 || { tail -20 gpurun_out/$TAG/$N.$R.log; exit 1; }
    grep '^{' gpurun_out/$TAG/$N.$R.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$N', round(d['ms_per_step'],2), round(d['value']/1e9,2), d['config'].get('step_overlap'), d.get('cpu_baseline', {}).get('sample_check', {}).get('identical'))"
  done
done
