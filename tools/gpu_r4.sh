#!/bin/bash
# Round-4 GPU session steps (each bounded, stop at the first failure):
#   tests    the -m gpu suite (PYTEST_ARGS narrows it)
#   tok      tokenizer timing of the tree's library and of LIBS (ab/lib_*.so) on MB of text
#   bench    bench.py with BENCH_ARGS (default: no CPU baseline, no front-end leg)
#   benchmat the same with --rows materialize
#   kt       rocprofv3 kernel trace of a 2-step bench (BENCH_ARGS)
#   TAG=x STEPS="tests tok bench" LIBS="ab/lib_head.so" bash tools/gpu_r4.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r4}; mkdir -p $OUT
export TMPDIR=/tmp
BA=${BENCH_ARGS:-"--no-cpu-baseline --frontend-mb 0"}
for S in ${STEPS:-tests tok bench}; do
  case $S in
    tests)
      timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "Error|FAILED|assert" $OUT/pytest_gpu.log | head -30; tail -5 $OUT/pytest_gpu.log; exit 1; }
      tail -1 $OUT/pytest_gpu.log ;;
    tok)
      for L in lddl_amd/liblddl_amd.so ${LIBS}; do
        N=$(basename $L .so)
        LDDL_LIB=$PWD/$L timeout -k 10 300 python -u tools/tok_check.py ${MB:-2048} 5 > $OUT/tok_$N.log 2>&1 || { echo "tok $N failed"; tail $OUT/tok_$N.log; exit 1; }
        echo "== $N"; grep -v "amdgpu.ids\|^gen" $OUT/tok_$N.log
      done ;;
    bench|benchmat)
      X=""; [ $S = benchmat ] && X="--rows materialize"
      timeout -k 10 600 python -u bench.py $BA $X > $OUT/$S.log 2>&1 || { echo "$S failed"; tail -20 $OUT/$S.log; exit 1; }
      tail -1 $OUT/$S.log > $OUT/$S.json
      python3 -c "import json; d=json.load(open('$OUT/$S.json')); print('$S', round(d['ms_per_step'],1), 'ms/step', round(d['value']/1e9,2), 'G tok/s', 'tok', {k: round(v,1) for k,v in d['tokenize_kernels_ms'].items()}, 'writer rows/s', round(d.get('parquet_writer',{}).get('rows_per_s',0)))" ;;
    kt|kthead)
      # kthead: the same trace with LDDL_LIB=KTLIB (default ab/lib_head.so) and materialised rows
      X=""; E=""; [ $S = kthead ] && { X="--rows materialize"; E="LDDL_LIB=$PWD/${KTLIB:-ab/lib_head.so}"; }
      env $E timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/$S -o kt --output-format csv -- python -u bench.py $BA --frontend-mb 0 $X --parquet-parts 0 --steps 2 --warmup 1 > $OUT/$S.log 2>&1 || { echo "kernel trace failed"; tail -20 $OUT/$S.log; exit 1; }
      f=$(find $OUT/$S -name '*kernel_stats.csv' | head -1); cp $f $OUT/${S}_stats.csv
      echo "== $S"; cut -d, -f1-4 $OUT/${S}_stats.csv | head -14 ;;
    stamps)
      LDDL_TOK_DEBUG=1 NOCHECK=1 timeout -k 10 200 python tools/tok_check.py 1024 5 > $OUT/stamps.log 2>&1 || { echo "stamps failed"; tail $OUT/stamps.log; exit 1; }
      grep dbg $OUT/stamps.log | tail -1 ;;
  esac
done
