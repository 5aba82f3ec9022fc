#!/bin/bash
# The scan's two-choice whole-word table (LDDL_SCAN_TABLE=1) against the
# default vt-bucket probe (0): tokenizer GPU tests, tools/tok_check.py timing
# alternating, one FETCH_SIZE pass of a 1 GB tok_check each.
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5st}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_tokenize_gpu.py tests/test_boundary_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0 1 0; do
  LDDL_SCAN_TABLE=$v timeout -k 10 300 python -u tools/tok_check.py 1024 5 > $O/tok_$v.txt 2>&1 || { tail -5 $O/tok_$v.txt; exit 1; }
  echo "scan_table=$v $(grep -h 'per kernel' $O/tok_$v.txt) $(grep -h '^variant' $O/tok_$v.txt)" >> $O/summary.txt
done
for v in 1 0; do
  NOCHECK=1 LDDL_SCAN_TABLE=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/f$v -o pmc --output-format csv -- python -u tools/tok_check.py 1024 5 > $O/f$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $O/f$v.log; exit 1; }
  f=$(find $O/f$v -name '*counter_collection.csv' | head -1)
  python3 - "$f" "$v" >> $O/summary.txt <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
  if 'scan_kernel' in r['Kernel_Name'] and r['Counter_Name'] == 'FETCH_SIZE':
    acc[r['Dispatch_Id']].append(float(r['Counter_Value']))
vals = [sum(v) for v in acc.values()]
print('scan_table=%s scan FETCH_SIZE per dispatch (KB, raw): mean %.4g over %d dispatches' % (sys.argv[2], sum(vals) / max(1, len(vals)), len(vals)))
PY
done
cat $O/summary.txt
