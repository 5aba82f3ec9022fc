#!/bin/bash
# GPU session: the -m gpu suite (SKIP_TESTS=1 skips it), then the tokenizer
# A/B of the working tree's library against LIBS (ab/lib_*.so, tools/ab_head.sh)
# on MB of synthetic Wikipedia-style text, each with VARIANTS (tok_check.py
# algo[:cfg] list, default "5").
#   TAG=r3_x LIBS="ab/lib_head.so" VARIANTS="5 5:1" MB=1024 tools/gpu_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-gpu_ab}; mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "Error|FAILED|assert" $OUT/pytest_gpu.log | head -30; tail -5 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
for L in lddl_amd/liblddl_amd.so ${LIBS}; do
  N=$(basename $L .so)
  LDDL_LIB=$PWD/$L timeout -k 10 300 python -u tools/tok_check.py ${MB:-1024} ${VARIANTS:-5} > $OUT/$N.log 2>&1 || { echo "$N failed"; tail $OUT/$N.log; exit 1; }
  echo "== $N"; grep -v "amdgpu.ids\|^gen" $OUT/$N.log
done
