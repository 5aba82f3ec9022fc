#!/bin/bash
# expand_kernel grid A/B (blocks per CU, LDDL_EXP_BLOCKS) on 2 GiB with
# tools/tok_check.py (min of 3, kernel times from its HIP events), one call.
#   TAG=r4_exp bash tools/r4_exp.sh
set -o pipefail
O=gpurun_out/${TAG:-r4_exp}
mkdir -p $O
for b in ${BLOCKS:-8 10 12 16}; do
  LDDL_EXP_BLOCKS=$b timeout -k 10 300 python -u tools/tok_check.py 2048 > $O/tok_$b.log 2>&1 || { tail -5 $O/tok_$b.log; exit 1; }
  echo "== blocks $b: $(grep -v amdgpu.ids $O/tok_$b.log | tail -3 | tr '\n' ' ')"
done
