#!/bin/bash
# wp_kernel A/B: tools/tok_check.py 2048 (parity against the oracle + per-kernel times, min of 3) for the
# tree's library and LIBS, then the tokenizer GPU tests on the tree.
#   TAG=r4_wp LIBS="ab/lib_base.so" bash tools/r4_wp.sh
set -o pipefail
O=gpurun_out/${TAG:-r4_wp}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_tokenize_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for LIB in tree $LIBS tree; do
  N=$(basename $LIB .so)
  if [ $LIB = tree ]; then unset LDDL_LIB; else export LDDL_LIB=$(realpath $LIB); fi
  timeout -k 10 300 python -u tools/tok_check.py 2048 > $O/tok_$N.log 2>&1 || { tail -5 $O/tok_$N.log; exit 1; }
  echo "== $N: $(grep -v amdgpu.ids $O/tok_$N.log | grep -E 'per kernel|variant' | tr '\n' ' ')"
done
