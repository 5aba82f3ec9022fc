#!/bin/bash
# Round 6: the bench step at tokenizer segment sizes (LDDL_SPLIT_SEG, tiles of
# 1 KiB; default 4 Mi = 4 GiB, 5 launches per 21.4 GB step), alternating.
#   Usage: SEGS="4194304 8388608" bash tools/r6_seg.sh TAG
set -o pipefail
TAG=${1:-r6seg}
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out/$TAG
B="bench.py --cpu-seconds 2 --parquet-parts 0 --frontend-mb 0 --frontend-c2-mb 0 --legs none --steps ${STEPS:-3} --warmup 1"
for R in 1 2; do
  for S in ${SEGS:-4194304 8388608}; do
    LDDL_SPLIT_SEG=$S timeout -k 10 400 python -u $B > gpurun_out/$TAG/seg$S.$R.log 2>&1 || { tail -20 gpurun_out/$TAG/seg$S.$R.log; exit 1; }
    grep '^{' gpurun_out/$TAG/seg$S.$R.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('seg $S', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['tokenize_kernels_ms'].items()}, d['roofline']['launches_per_step'], d.get('cpu_baseline',{}).get('sample_check',{}).get('identical'))"
  done
done
