#!/usr/bin/env python3
"""Golden vectors for the load balancer, produced by the REFERENCE's own
lddl/dask/load_balance.py main() (run HERE only; /root/reference is read,
never copied).

mpi4py is absent in this image; load_balance only needs COMM_WORLD's size /
rank / barrier / in-place Allreduce, so a one-rank communicator is injected
(with one rank every Allreduce is the identity and rank 0 does all IO, which
is what every rank's files look like in a multi-rank run too: the rank only
decides who reads/writes a table, not which rows go where).

Input: parquet files whose single int64 column 'rid' = file_index << 32 | row.
Output (data only): tests/golden/balance.json.gz -- per case the input file
names and row counts, --num-shards, and per written shard file its rows as
(file_index, first_row, n) runs, plus the .num_samples.json the reference wrote.
"""
import gzip
import json
import os
import sys
import tempfile
import types

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Comm:
  def Get_size(self):
    return 1

  def Get_rank(self):
    return 0

  def barrier(self):
    return None

  def Allreduce(self, sendbuf, recvbuf, op=None):
    return None  # in place, one rank


mpi = types.ModuleType('mpi4py.MPI')
mpi.COMM_WORLD = _Comm()
mpi.SUM = 'sum'
mpi.IN_PLACE = object()
pkg = types.ModuleType('mpi4py')
pkg.MPI = mpi
sys.modules['mpi4py'] = pkg
sys.modules['mpi4py.MPI'] = mpi
sys.path.insert(0, '/root/reference')
if not hasattr(np, 'NAN'):
  np.NAN = np.nan  # numpy 2 dropped the alias the reference's log line uses (load_balance.py:262)
import lddl.dask.load_balance as ref  # noqa: E402

# The reference never terminates when the total is divisible by --num-shards
# and some shard passes through exactly base+1 samples (Progress keeps a
# zero-count base+1 target, load_balance.py:163-167,190-197: that shard is
# taken as ready, the rest can no longer pair up).  Such cases are recorded
# as 'hang' instead of rows.
_report = ref.Progress.report


def _bounded_report(self, shards):
  self._n_reports = getattr(self, '_n_reports', 0) + 1
  if self._n_reports > 1000:
    raise TimeoutError('reference load balancer does not terminate')
  return _report(self, shards)


ref.Progress.report = _bounded_report


def runs(rid):
  """int64 rid column -> [(file, first_row, n)] runs"""
  out = []
  for v in rid:
    f, r = int(v) >> 32, int(v) & 0xFFFFFFFF
    if out and out[-1][0] == f and out[-1][1] + out[-1][2] == r:
      out[-1][2] += 1
    else:
      out.append([f, r, 1])
  return out


def case(rng, names, counts, num_shards, bin_ids=None):
  with tempfile.TemporaryDirectory() as d:
    ind, outd = os.path.join(d, 'in'), os.path.join(d, 'out')
    os.makedirs(ind)
    for i, (nm, n) in enumerate(zip(names, counts)):
      rid = (np.int64(i) << 32) + np.arange(n, dtype=np.int64)
      pq.write_table(pa.table({'rid': rid}), os.path.join(ind, nm))
    args = types.SimpleNamespace(indir=ind, outdir=outd, num_shards=num_shards, bin_ids=bin_ids, keep_orig=True)
    import contextlib
    import io
    try:
      with contextlib.redirect_stdout(io.StringIO()):
        ref.main(args)
    except (TimeoutError, TypeError) as e:
      # TypeError: more shards than files leaves Shard._input_files None
      # (load_balance.py:240-242), which flush() / _load() cannot take
      return {'files': names, 'counts': [int(c) for c in counts], 'num_shards': num_shards, 'bin_ids': bin_ids,
              'error': type(e).__name__}
    shards = {}
    for f in sorted(os.listdir(outd)):
      if f.startswith('shard-'):
        shards[f] = runs(pq.read_table(os.path.join(outd, f)).column('rid').to_numpy())
    with open(os.path.join(outd, '.num_samples.json')) as f:
      ns = json.load(f)
  return {'files': names, 'counts': [int(c) for c in counts], 'num_shards': num_shards, 'bin_ids': bin_ids,
          'shards': shards, 'num_samples': ns, 'error': None}


def main():
  rng = np.random.default_rng(20261016)
  cases = []
  # unbinned: part.{i}.parquet, lexicographic file order (part.10 < part.2)
  for n_files, num_shards, hi in [(1, 1, 50), (5, 3, 40), (12, 4, 100), (12, 7, 30), (30, 8, 500), (9, 9, 20),
                                  (20, 5, 3), (16, 16, 64)]:
    names = ['part.%d.parquet' % i for i in range(n_files)]
    counts = rng.integers(0, hi, n_files)
    cases.append(case(rng, names, counts, num_shards))
  for seed in range(40):  # random small cases
    n_files, num_shards = int(rng.integers(1, 25)), int(rng.integers(1, 12))
    names = ['part.%d.parquet' % i for i in range(n_files)]
    cases.append(case(rng, names, rng.integers(0, int(rng.integers(1, 200)), n_files), num_shards))
  # equal counts (total divisible: the targets dict keeps a zero entry)
  cases.append(case(rng, ['part.%d.parquet' % i for i in range(6)], [10] * 6, 3))
  cases.append(case(rng, ['part.%d.parquet' % i for i in range(6)], [10] * 6, 4))
  # binned: part.{i}.parquet_{b}, every bin present for every partition
  for n_part, nbins, num_shards, hi in [(6, 4, 3, 30), (11, 8, 4, 60), (7, 2, 5, 10), (3, 2, 5, 10)]:
    names = ['part.%d.parquet_%d' % (p, b) for p in range(n_part) for b in range(nbins)]
    counts = rng.integers(0, hi, len(names))
    cases.append(case(rng, names, counts, num_shards))
  out = {'generator': 'tools/gen_golden_balance.py', 'reference': 'lddl/dask/load_balance.py:129-369',
         'cases': cases}
  path = os.path.join(ROOT, 'tests', 'golden', 'balance.json.gz')
  with gzip.open(path, 'wt') as f:
    json.dump(out, f)
  print(path, len(cases), 'cases')


if __name__ == '__main__':
  main()
