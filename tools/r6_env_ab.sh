#!/bin/bash
# Round 6: headline bench step under environment variants, alternating
# (each variant "NAME=VALUE", "-" = none), two rounds.
#   Usage: VARIANTS="- LDDL_EXP_BLOCKS=8 LDDL_EXP_BLOCKS=24" bash tools/r6_env_ab.sh TAG
set -o pipefail
TAG=${1:-r6env}
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out/$TAG
B="bench.py --no-cpu-baseline --no-sample-check --parquet-parts 0 --frontend-mb 0 --frontend-c2-mb 0 --legs none --steps ${STEPS:-3} --warmup 1"
for R in 1 2; do
  for V in ${VARIANTS:--}; do
    N=$(echo "$V" | tr '=' '_')
    if [ "$V" = "-" ]; then E=""; else E="$V"; fi
    env $E timeout -k 10 400 python -u $B > gpurun_out/$TAG/$N.$R.log 2>&1 || { tail -20 gpurun_out/$TAG/$N.$R.log; exit 1; }
    grep '^{' gpurun_out/$TAG/$N.$R.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$N', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['tokenize_kernels_ms'].items()})"
  done
done
