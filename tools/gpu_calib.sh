#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes over tools/fetch_calib (see its header).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-calib}
mkdir -p $OUT
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $C -d $OUT/pmc_$C -o pmc --output-format csv -- ./tools/fetch_calib > $OUT/$C.log 2>&1 || { echo "pass $C failed"; exit 1; }
  python - $OUT/pmc_$C <<'PY'
import csv, glob, sys, collections
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
  per = collections.defaultdict(float)
  for r in csv.DictReader(open(f)):
    per[(r['Dispatch_Id'], r['Kernel_Name'][:40], r['Counter_Name'])] += float(r['Counter_Value'])
  for k, v in sorted(per.items()): print(k, '%.6g KB' % v)
PY
done
