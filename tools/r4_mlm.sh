#!/bin/bash
# Masked path check: the pack / writer GPU tests, then a kernel trace of the
# 20 GB --masking bench step (masked packer, masked_lm_spans, row spans).
#   TAG=r4_mlm bash tools/r4_mlm.sh
set -o pipefail
O=gpurun_out/${TAG:-r4_mlm}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_pack_gpu.py tests/test_writer_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python -u bench.py --masking \
  --no-cpu-baseline --parquet-parts 0 --frontend-mb 0 --no-sample-check --steps 2 --warmup 1 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
tail -1 $O/kt.log > $O/bench.json
f=$(find $O/kt -name '*kernel_stats.csv' | head -1); cp $f $O/kernel_stats.csv
python3 -c "import json; d=json.load(open('$O/bench.json')); print('masked', round(d['ms_per_step'], 1), 'ms/step')"
grep -E "pack_bert_wave|masked_lm|rowspan" $O/kernel_stats.csv | cut -c1-150
