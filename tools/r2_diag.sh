#!/bin/bash
# Diagnostics: tokenizer phase stamps (LDDL_TOK_DEBUG=1) on a synthetic
# corpus, the masked packer's phase stamps and a masked-bench kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r2_diag}; mkdir -p $OUT
export TMPDIR=/tmp
LDDL_TOK_DEBUG=1 timeout -k 10 300 python -u tools/tok_check.py ${MB:-512} 5 > $OUT/tok_dbg.log 2>&1 || { tail $OUT/tok_dbg.log; exit 1; }
grep -v amdgpu.ids $OUT/tok_dbg.log | tail -6
[ -n "$SKIP_MASK" ] && exit 0
LDDL_PACK_DEBUG=1 timeout -k 10 600 python -u bench.py --masking --no-cpu-baseline --parquet-parts 0 --steps 1 --warmup 1 > $OUT/mask_dbg.log 2>&1 || { tail $OUT/mask_dbg.log; exit 1; }
grep "pack dbg" $OUT/mask_dbg.log | tail -1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/mkt -o kt --output-format csv -- python -u bench.py --masking --no-cpu-baseline --parquet-parts 0 --steps 2 --warmup 1 > $OUT/mkt.log 2>&1 || { tail $OUT/mkt.log; exit 1; }
tail -1 $OUT/mkt.log | cut -c1-300
f=$(find $OUT/mkt -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 $f | head -12
