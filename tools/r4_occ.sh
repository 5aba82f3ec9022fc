#!/bin/bash
# Packer occupancy at the bench workload: LDDL_PACK_WAVES_CU caps the
# one-wave blocks per CU by padding the packer's dynamic LDS (20 412
# partitions = 2.5 rounds of 8 192 wave slots at 8 waves/SIMD, 3.3 rounds of
# 6 144 at 6).  Unmasked: default (32/CU, SGPR-bound), 28, 24; masked:
# default (24/CU), 20.  Alternating, fresh processes.
#   TAG=r4_occ bash tools/r4_occ.sh
set -o pipefail
O=gpurun_out/${TAG:-r4_occ}
mkdir -p $O
B="bench.py --no-cpu-baseline --parquet-parts 0 --frontend-mb 0 --no-sample-check"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_pack_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # tag, waves, extra bench args
  LDDL_PACK_WAVES_CU=$2 timeout -k 10 300 python -u $B $3 > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }
  python -c "
import json; d = json.loads(open('$O/$1.log').read().strip().splitlines()[-1])
print('$1', round(d['ms_per_step'], 2), 'ms/step', 'tokenize', round(d['tokenize_ms'], 2))"
}
for i in 1 2; do
  run u_def_$i 0 "--steps 8 --warmup 2" && run u_28_$i 28 "--steps 8 --warmup 2" && run u_24_$i 24 "--steps 8 --warmup 2" || exit 1
done
for i in 1 2; do
  run m_def_$i 0 "--masking --steps 4 --warmup 1" && run m_20_$i 20 "--masking --steps 4 --warmup 1" || exit 1
done
