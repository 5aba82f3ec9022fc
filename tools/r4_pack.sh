#!/bin/bash
# Front-end cProfile + BERT packer phase stamps (GPU box):
#   TAG=r4_pack bash tools/r4_pack.sh
# fep/prof.txt: tools/frontend_prof.py 100 (the bench front-end leg's flags)
# stamps.log: bench.py --steps 1 with LDDL_PACK_DEBUG=1 (the [lddl pack dbg]
#   line: per-phase s_memtime ticks summed over the partitions' waves)
set -o pipefail
O=gpurun_out/${TAG:-r4_pack}
mkdir -p $O/fep
timeout -k 10 300 python -u tools/frontend_prof.py 100 > $O/fep/prof.txt 2>&1 &&
LDDL_PACK_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --frontend-mb 0 --no-cpu-baseline \
  --no-sample-check --parquet-parts 0 ${BENCH_ARGS} > $O/stamps.log 2>&1
