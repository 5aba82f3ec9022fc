#!/bin/bash
# bench.py variants at 1 GB per GPU with the host leg (cpu baseline +
# sampled-partition oracle check): wiki, code, masking, wikibooks.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_bvar}; mkdir -p $OUT
IFS=";" read -ra VS <<< "${VARIANTS:---corpus wiki;--corpus code;--masking;--corpus wikibooks}"
for V in "${VS[@]}"; do
  N=$(echo $V | tr -d ' -')
  timeout -k 10 900 python -u bench.py --corpus-gb ${GB:-1} ${EXTRA:---steps 1 --warmup 1 --cpu-seconds 4 --parquet-parts 4} $V > $OUT/$N.log 2>&1 || { echo "bench $V failed"; tail -20 $OUT/$N.log; exit 1; }
  tail -1 $OUT/$N.log > $OUT/$N.json
  tail -1 $OUT/$N.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu_baseline',{}); print('$N', round(d['value']/1e9,2), 'Gtok/s', 'check', c.get('sample_check'), 'ref', (c.get('reference_library') or {}).get('value'))"
done
