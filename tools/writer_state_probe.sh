#!/bin/bash
# Writer sample (bench.py, no CLI legs) on a fresh box, then after 8 s of
# 16 busy processes (CPU only, no file I/O), then again: does a CPU-heavy
# stage leave later writer samples slower?  CPU MHz read around each step.
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5wstate}; mkdir -p $O
mhz() { awk '/cpu MHz/ {s+=$4; n++} END {printf "%.0f", s/n}' /proc/cpuinfo; }
run() {
  timeout -k 10 300 python -u bench.py --legs none --no-cpu-baseline --no-sample-check --steps 1 --warmup 1 --frontend-mb 0 --frontend-c2-mb 0 > $O/b.json 2>> $O/err.log || exit 1
  grep -h "^{" $O/b.json | python3 -c "import json,sys; p=json.load(sys.stdin)['parquet_writer']; print('$1', 'writer', round(p['rows_per_s']/1e6,3), 'M rows/s, table_s', round(p['stages']['table_s'],3))" >> $O/summary.txt
  echo "  mean cpu MHz $(mhz)" >> $O/summary.txt
}
echo "start mean cpu MHz $(mhz)" > $O/summary.txt
run fresh1
run fresh2
timeout -k 5 30 python3 -c "
import multiprocessing as mp, time
def burn(_):
  t = time.time(); x = 0
  while time.time() - t < 8: x += 1
  return x
with mp.Pool(16) as p: p.map(burn, range(16))
" || exit 1
echo "after burn mean cpu MHz $(mhz)" >> $O/summary.txt
run after_burn1
run after_burn2
cat $O/summary.txt
