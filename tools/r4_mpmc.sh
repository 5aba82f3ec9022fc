#!/bin/bash
# Masked packer counters: SQ instruction mix and waits of a 1-step --masking bench (two passes).
#   TAG=r4_mpmc bash tools/r4_mpmc.sh
set -o pipefail
O=gpurun_out/${TAG:-r4_mpmc}
mkdir -p $O
export TMPDIR=/tmp
B="bench.py --masking --no-cpu-baseline --parquet-parts 0 --frontend-mb 0 --no-sample-check --steps 1 --warmup 0"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/p1 -o pmc --output-format csv -- python -u $B > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/p2 -o pmc --output-format csv -- python -u $B > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $O/p3 -o pmc --output-format csv -- python -u $B > $O/p3.log 2>&1 || { tail -5 $O/p3.log; exit 1; }
python tools/pmc_summary.py $O > $O/pmc_summary.txt
grep -A20 "pack_bert_wave_kernel<1" $O/pmc_summary.txt | head -22
