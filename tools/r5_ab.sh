#!/bin/bash
# Round 5 A/B: tools/tok_check.py (variant 5) with the working tree's library
# and each LIBS entry (ab/lib_*.so, tools/ab_build.py), in one call.
#   LIBS="ab/lib_x.so ab/lib_y.so" bash tools/r5_ab.sh TAG [MB]
set -o pipefail
TAG=${1:-r5ab}; MB=${2:-1024}
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out/$TAG
for L in lddl_amd/liblddl_amd.so ${LIBS}; do
  N=$(basename $L .so)
  LDDL_LIB=$PWD/$L timeout -k 10 300 python -u tools/tok_check.py $MB ${VARIANT:-5} > gpurun_out/$TAG/$N.txt 2>&1 || { tail -5 gpurun_out/$TAG/$N.txt; exit 1; }
done
