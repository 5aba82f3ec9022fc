#!/bin/bash
# rocprofv3 kernel trace + PMC passes of the bench command (each bounded).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-prof}
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python $B > $OUT/kt.log 2>&1 && echo "kt ok" &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o pmc --output-format csv -- python $B > $OUT/pmc_fetch.log 2>&1 && echo "fetch ok" &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o pmc --output-format csv -- python $B > $OUT/pmc_write.log 2>&1 && echo "write ok" &&
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/pmc_sq -o pmc --output-format csv -- python $B > $OUT/pmc_sq.log 2>&1 && echo "sq ok"
tail -1 $OUT/kt.log
