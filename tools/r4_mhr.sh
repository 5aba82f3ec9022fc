#!/bin/bash
# masked packer tests (high ratio: MASK = 1 at its pick capacity, MASK = 2 fallback)
set -o pipefail
O=gpurun_out/${TAG:-r4_mhr}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_pack_gpu.py -k "masked" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest.log | tail -20
