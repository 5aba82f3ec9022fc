#!/bin/bash
# A/B of packer builds in one GPU call: for each library (the tree's and
# LIBS=ab/lib_*.so), a kernel trace of a 2-step bench and an SQ_INSTS_SALU pass.
#   TAG=r4_ab LIBS="ab/lib_a.so ab/lib_b.so" bash tools/r4_ab.sh
set -o pipefail
O=gpurun_out/${TAG:-r4_ab}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then  # the tree's pack GPU tests first
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $TESTS > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
B="bench.py --no-cpu-baseline --parquet-parts 0 --frontend-mb 0 --no-sample-check"
for LIB in tree $LIBS; do
  N=$(basename $LIB .so)
  if [ $LIB = tree ]; then unset LDDL_LIB; else export LDDL_LIB=$(realpath $LIB); fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$N -o kt --output-format csv -- python -u $B --steps 2 --warmup 1 > $O/kt_$N.log 2>&1 || { tail -20 $O/kt_$N.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU -d $O/p_$N -o pmc --output-format csv -- python -u $B --steps 1 --warmup 0 > $O/p_$N.log 2>&1 || { tail -5 $O/p_$N.log; exit 1; }
  f=$(find $O/kt_$N -name '*kernel_stats.csv' | head -1)
  echo "== $N: $(grep pack_bert_wave $f | cut -d, -f2-4)"
  python3 - $O/p_$N <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
  for r in csv.DictReader(open(f)):
    if 'pack_bert_wave' in r['Kernel_Name']:
      agg[r['Counter_Name']] += float(r['Counter_Value'])
print({k: '%.4g' % v for k, v in agg.items()})
PY
done
if [ -n "$MASK_STAMPS" ]; then  # masked packer phase stamps of the tree
  unset LDDL_LIB
  LDDL_PACK_DEBUG=1 timeout -k 10 300 python -u bench.py --masking --steps 1 --warmup 0 --no-cpu-baseline --frontend-mb 0 \
    --parquet-parts 0 --no-sample-check > $O/mask_stamps.log 2>&1 || { tail -5 $O/mask_stamps.log; exit 1; }
  grep "pack dbg" $O/mask_stamps.log | head -1
fi
