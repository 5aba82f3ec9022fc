#!/bin/bash
# tokenizer-only PMC passes (each bounded); results under gpurun_out/$TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-proftok}
mkdir -p $OUT
export TMPDIR=/tmp
MB=${MB:-128}
python - <<'PY' > $OUT/copy.txt 2>&1
import torch, time
a = torch.empty(256 << 20, dtype=torch.uint8, device='cuda'); b = torch.empty_like(a)
for _ in range(3): b.copy_(a)
torch.cuda.synchronize(); s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
s.record(); [b.copy_(a) for _ in range(10)]; e.record(); torch.cuda.synchronize()
ms = s.elapsed_time(e) / 10
print('copy 256MB: %.3f ms  %.1f GB/s (r+w)' % (ms, 2 * 256 * 1.048576 / ms))
PY
cat $OUT/copy.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python tools/tok_perf.py $MB > $OUT/kt.log 2>&1 && echo kt ok &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/pmc1 -o pmc --output-format csv -- python tools/tok_perf.py $MB > $OUT/pmc1.log 2>&1 && echo pmc1 ok &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_FLAT -d $OUT/pmc2 -o pmc --output-format csv -- python tools/tok_perf.py $MB > $OUT/pmc2.log 2>&1 && echo pmc2 ok &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc3 -o pmc --output-format csv -- python tools/tok_perf.py $MB > $OUT/pmc3.log 2>&1 && echo pmc3 ok &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc4 -o pmc --output-format csv -- python tools/tok_perf.py $MB > $OUT/pmc4.log 2>&1 && echo pmc4 ok
