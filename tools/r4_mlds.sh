#!/bin/bash
# Masked packer with the seq <= 512 masking lists at 4.5 KB of LDS (32
# one-wave blocks per CU): pack / writer / collate GPU tests on the tree,
# then the masked bench step alternating the tree and LIB (the previous
# library), fresh processes.
#   TAG=r4_mlds LIB=ab/lib_base.so bash tools/r4_mlds.sh
set -o pipefail
O=gpurun_out/${TAG:-r4_mlds}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_pack_gpu.py tests/test_writer_gpu.py tests/test_collate_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="bench.py --masking --no-cpu-baseline --parquet-parts 0 --frontend-mb 0 --steps 4 --warmup 1"
for i in 1 2; do
  for v in tree base; do
    if [ $v = base ]; then export LDDL_LIB=$(realpath $LIB); else unset LDDL_LIB; fi
    timeout -k 10 300 python -u $B > $O/m_${v}_$i.log 2>&1 || { tail -5 $O/m_${v}_$i.log; exit 1; }
    python -c "
import json; d = json.loads(open('$O/m_${v}_$i.log').read().strip().splitlines()[-1])
print('$v', round(d['ms_per_step'], 2), 'ms/step', d.get('sample_check', d.get('cpu_baseline', {}).get('sample_check')))"
  done
done
unset LDDL_LIB
# one full-size masked partition of the tree's run against the oracle
timeout -k 10 400 python -u bench.py --masking --parquet-parts 0 --frontend-mb 0 --steps 1 --warmup 0 > $O/m_check.log 2>&1 || { tail -5 $O/m_check.log; exit 1; }
python -c "
import json; d = json.loads(open('$O/m_check.log').read().strip().splitlines()[-1]); print('sample check', d['cpu_baseline']['sample_check'])"
