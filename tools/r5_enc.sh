set -o pipefail
O=gpurun_out/r5enc1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_writer_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for C in wiki code; do for V in 1 0 1 0; do
  LDDL_ENCODE_PROCS=$V timeout -k 10 300 python -u bench.py --corpus $C --steps 1 --legs none --frontend-mb 0 --frontend-c2-mb 0 --no-cpu-baseline --no-sample-check > $O/${C}_$V.json 2> $O/${C}_$V.err || { tail -5 $O/${C}_$V.err; exit 1; }
  grep "^{" $O/${C}_$V.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['parquet_writer']; print('$C procs=$V', round(p['rows_per_s']/1e6,3), 'M rows/s', p.get('encoder'), {k: round(v,3) for k,v in p['stages'].items()})" | tee -a $O/summary.txt
done; done
timeout -k 10 600 python -u bench.py --legs none > $O/full.json 2> $O/full.err || { tail -5 $O/full.err; exit 1; }
grep "^{" $O/full.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('full', d['ms_per_step'], d['parquet_writer']['rows_per_s'], {k: d['frontend_c2'][k] for k in ('seconds','raw_mb_per_s','gpu_init_s','write_s','gpu_s','host_split_s')}, {k: d['frontend'][k] for k in ('seconds','raw_mb_per_s','write_s')})" | tee -a $O/summary.txt
