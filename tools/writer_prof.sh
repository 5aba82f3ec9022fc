#!/bin/bash
# cProfile of bench.py's parquet-writer leg (CodeBERT and BERT), small corpus
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-writer_prof}
mkdir -p $OUT
for C in code wiki; do
  timeout -k 10 300 python -u -m cProfile -o $OUT/$C.prof bench.py --corpus $C --corpus-gb 2 --steps 1 --warmup 0 \
    --no-cpu-baseline --frontend-mb 0 --no-sample-check > $OUT/$C.log 2>&1 || { echo "$C failed"; tail -20 $OUT/$C.log; exit 1; }
  python -c "
import pstats,json
l=open('$OUT/$C.log').read().strip().splitlines()[-1]
print('$C', json.loads(l)['parquet_writer'])
s=pstats.Stats('$OUT/$C.prof'); s.sort_stats('cumulative').print_stats('writer|pyarrow|parquet|numpy|render|row_docs|take|array', 30)
" > $OUT/$C.txt 2>&1
  head -3 $OUT/$C.txt
done
