#!/bin/bash
# Packer occupancy timeline (LDDL_PACK_DEBUG=1: per-wave start / end on the
# 100 MHz device clock, summarised by capi as "[lddl pack tl]") of a 1-step
# bench, masked seq 512 / 128 and unmasked seq 512, at the resident-wave caps
# in CUS (LDDL_PACK_WAVES_CU; 0 = the kernel's own occupancy).
#   TAG=r6_tl [LIBS=...] [CFGS="m512 m128 u512"] [CUS="0"] [ORDERS="1"] [TESTS=1] bash tools/r6_tl.sh
# ORDERS: LDDL_PACK_ORDER values (1 = longest-first dispatch, 0 = blockIdx order); TESTS=1 first runs the
# packer GPU tests.
set -o pipefail
O=gpurun_out/${TAG:-r6_tl}
mkdir -p $O
export TMPDIR=/tmp
B="bench.py --no-cpu-baseline --parquet-parts 0 --frontend-mb 0 --frontend-c2-mb 0 --legs none --no-sample-check --steps 1 --warmup 1"
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -rs -m gpu -k "pack or mask or row or bench or boundary" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for L in ${LIBS:-lddl_amd/liblddl_amd.so}; do
  N=$(basename $L .so)
  for K in ${CFGS:-m512 m128 u512}; do
    case $K in m512) A="--masking --target-seq-length 512";; m128) A="--masking --target-seq-length 128";; *) A="--target-seq-length 512";; esac
    for W in ${CUS:-0}; do
    for R in ${ORDERS:-1}; do
      F=$O/${N}_${K}_w${W}_o$R
      LDDL_PACK_ORDER=$R LDDL_PACK_WAVES_CU=$W LDDL_LIB=$PWD/$L LDDL_PACK_DEBUG=1 timeout -k 10 300 python -u $B $A > $F.log 2>&1 || { tail -5 $F.log; exit 1; }
      LDDL_PACK_ORDER=$R LDDL_PACK_WAVES_CU=$W LDDL_LIB=$PWD/$L timeout -k 10 300 python -u $B $A --steps 3 > $F.t.log 2>&1 || { tail -5 $F.t.log; exit 1; }
      echo "$N $K w$W order$R: $(python3 -c "import json; d=json.loads([l for l in open('$F.t.log') if l.startswith('{')][-1]); print(round(d['ms_per_step'],1), 'ms/step')")"
      grep -h 'lddl pack tl' $F.log | tail -2
    done
    done
  done
done
