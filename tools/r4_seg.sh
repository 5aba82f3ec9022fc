#!/bin/bash
# Tokenizer segment size at the bench workload: LDDL_SPLIT_SEG tiles (1 KiB)
# per segment -- 4 GiB (default, 5 launches per kernel per step), 8 GiB (3),
# 11 GiB (2) -- alternating, each a fresh bench process.
#   TAG=r4_seg bash tools/r4_seg.sh
set -o pipefail
O=gpurun_out/${TAG:-r4_seg}
mkdir -p $O
B="bench.py --no-cpu-baseline --parquet-parts 0 --frontend-mb 0 --no-sample-check --steps 10 --warmup 2"
for i in 1 2; do
  for seg in 4194304 8388608 11534336; do
    LDDL_SPLIT_SEG=$seg timeout -k 10 300 python -u $B > $O/b_${seg}_$i.log 2>&1 || { tail -5 $O/b_${seg}_$i.log; exit 1; }
    python -c "
import json; d = json.loads(open('$O/b_${seg}_$i.log').read().strip().splitlines()[-1])
print($seg, round(d['ms_per_step'], 2), 'ms/step', {k: round(v, 2) for k, v in d['tokenize_kernels_ms'].items()}, 'tok', round(d['tokenize_ms'], 2))"
  done
done
