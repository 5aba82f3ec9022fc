#!/bin/bash
# Packer + front-end check: the pack / writer / CLI GPU tests, a kernel
# trace and an SQ_INSTS_SALU pass of a 1-step bench (the packer's seconds and
# scalar work), then the front-end CLI timing per --chunk-mb, each in a fresh
# process (first-use costs included, as in bench.py's leg):
#   TAG=r4_fe [CHUNKS="16 32"] bash tools/r4_fe.sh
set -o pipefail
O=gpurun_out/${TAG:-r4_fe}
mkdir -p $O
export TMPDIR=/tmp
TESTS="tests/test_pack_gpu.py tests/test_writer_gpu.py tests/test_preprocess.py"
[ -n "$SKIP_PACK" ] && TESTS="tests/test_writer_gpu.py tests/test_preprocess.py"
[ -n "$SKIP_FE" ] && TESTS="tests/test_pack_gpu.py"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu $TESTS > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
if [ -n "$CODE_WRITER" ]; then
  timeout -k 10 300 python -u bench.py --corpus code --no-cpu-baseline --frontend-mb 0 --steps 1 --warmup 0 > $O/code.log 2>&1 || { tail -5 $O/code.log; exit 1; }
  tail -1 $O/code.log > $O/code.json
  python -c "import json; print('code writer', json.load(open('$O/code.json'))['parquet_writer'])"
fi
B="bench.py --no-cpu-baseline --parquet-parts 0 --frontend-mb 0 --no-sample-check"
[ -z "$SKIP_PACK" ] && { timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python -u $B --steps 2 --warmup 1 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
f=$(find $O/kt -name '*kernel_stats.csv' | head -1); cp $f $O/kernel_stats.csv
grep -E "pack_bert_wave|scan_kernel" $O/kernel_stats.csv | cut -c1-160
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVES -d $O/p1 -o pmc --output-format csv -- python -u $B --steps 1 --warmup 0 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
python tools/pmc_summary.py $O > $O/pmc_summary.txt; grep -A3 'pack_bert_wave' $O/pmc_summary.txt | head -4; }
[ -n "$SKIP_FE" ] && exit 0
for c in ${CHUNKS:-8 16 32 64}; do
  timeout -k 10 200 python -u -c "import bench, json; print(json.dumps(bench.frontend_leg(100, $c)))" \
    > $O/fe_$c.json 2> $O/fe_$c.err || { tail -5 $O/fe_$c.err; exit 1; }
done
grep -h raw_mb_per_s $O/fe_*.json | python -c "
import json, sys
for l in sys.stdin:
  d = json.loads(l)
  print(d['chunks'], 'chunks', round(d['raw_mb_per_s'], 1), 'MB/s', {k: round(d[k], 3) for k in ('seconds', 'host_split_s', 'split_wait_s', 'gpu_s', 'write_s', 'write_wait_s')})
"
