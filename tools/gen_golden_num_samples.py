#!/usr/bin/env python3
"""Golden vector for generate_num_samples_cache, produced by the REFERENCE's
own lddl/dask/load_balance.py:generate_num_samples_cache (:428-455, console
script `generate_num_samples_cache`, setup.py:72), run HERE only
(/root/reference is read, never copied).

mpi4py is absent in this image: a one-rank COMM_WORLD is injected, as in
tools/gen_golden_balance.py (with one rank the Allreduce of the per-file
counts is the identity).

Input: a directory tree of parquet files (balanced shards, binned and
unbinned names, a nested directory, a non-parquet file, an empty shard).
Output (data only): tests/golden/num_samples_cache.json -- the files as
(relative path, row count) and the exact text of the .num_samples.json the
reference wrote.
"""
import json
import os
import sys
import tempfile

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import gen_golden_balance  # noqa: E402,F401  (installs the one-rank mpi4py stub and imports the reference)
ref = sys.modules['lddl.dask.load_balance']

FILES = [('shard-0.parquet_0', 7), ('shard-1.parquet_0', 6), ('shard-0.parquet_1', 13), ('shard-1.parquet_1', 0),
         ('shard-10.parquet_0', 3), ('sub/shard-2.parquet_0', 5), ('part.3.parquet', 21), ('zz.parquet', 1)]
OTHER = ['notes.txt', '.num_samples.json.bak']


def make_tree(d, files=FILES, other=OTHER):
  for rel, n in files:
    p = os.path.join(d, rel)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    pq.write_table(pa.table({'A': pa.array(['a %d' % i for i in range(n)], pa.string()),
                             'num_tokens': pa.array(np.arange(n, dtype=np.uint16))}), p)
  for rel in other:
    with open(os.path.join(d, rel), 'w') as f:
      f.write('x\n')


def main():
  with tempfile.TemporaryDirectory() as d:
    make_tree(d)
    argv = sys.argv
    sys.argv = ['generate_num_samples_cache', '--indir', d]
    try:
      ref.generate_num_samples_cache()
    finally:
      sys.argv = argv
    text = open(os.path.join(d, '.num_samples.json')).read()
  out = os.path.join(ROOT, 'tests', 'golden', 'num_samples_cache.json')
  with open(out, 'w') as f:
    json.dump({'files': FILES, 'other': OTHER, 'num_samples_json': text}, f, indent=1)
  print(out, text)


if __name__ == '__main__':
  main()
