set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/sw
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tokenize_gpu.py tests/test_pack_gpu.py > gpurun_out/sw/pt.log 2>&1 || { tail -20 gpurun_out/sw/pt.log; exit 1; }
tail -1 gpurun_out/sw/pt.log
B="bench.py --no-cpu-baseline --no-sample-check --parquet-parts 0 --frontend-mb 0 --frontend-c2-mb 0 --legs none --steps 2 --warmup 1"
for L in lddl_amd/liblddl_amd.so ab/lib_swold.so; do
  N=$(basename $L .so)
  LDDL_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sw/$N -o kt --output-format csv -- python -u $B > gpurun_out/sw/$N.log 2>&1 || { tail -5 gpurun_out/sw/$N.log; exit 1; }
  f=$(find gpurun_out/sw/$N -name '*kernel_stats.csv' | head -1); cp $f gpurun_out/sw/${N}_stats.csv; grep -h 'scan_write\|scan_reduce' $f | cut -c1-110
done
