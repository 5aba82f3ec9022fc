#!/bin/bash
# Wave packer LDS-capacity sweep on the bench workload (pack kernel time from a kernel trace).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-packtune}
mkdir -p $OUT
export TMPDIR=/tmp
for caps in ${CAPS_LIST:-"0,0,0" "0,0,8192" "8192,512,0" "auto"}; do
  if [ "$caps" = auto ]; then unset LDDL_PACK_CAPS; else export LDDL_PACK_CAPS=$caps; fi
  d=$OUT/kt_${caps//,/_}
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d -o kt --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $d.log 2>&1 || { echo "caps $caps failed"; exit 1; }
  echo "caps $caps: $(python tools/pmc_summary.py $d | grep pack_bert)"
done
