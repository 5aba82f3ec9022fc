"""Parquet encode rate by sink and thread count on this host (no GPU):
the writer's host stage in isolation.  A synthetic table shaped like the
bench's seq-512 rows (~1.3 KB of A/B strings per row, is_random_next,
num_tokens, bin_id), 512 files of ~585 rows as writer.write_shards cuts
them, encoded with its settings (snappy, dictionary pages only for the
repeating columns) into: memory (pa.BufferOutputStream), files under
--dirs (e.g. /tmp and /dev/shm).
  python tools/pq_sink_probe.py [--threads 1,4,8,16] [--dirs /tmp,/dev/shm]"""
import argparse
import concurrent.futures as cf
import json
import os
import shutil
import tempfile
import time

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq


def table(n, avg, seed=0):
  rng = np.random.default_rng(seed)
  words = [bytes(rng.integers(97, 123, size=rng.integers(2, 10)).astype(np.uint8)) for _ in range(5000)]

  def col():
    k = np.maximum(1, rng.normal(avg / 6, avg / 24, size=n).astype(int))
    idx = rng.integers(0, 5000, size=int(k.sum()))
    parts, at = [], 0
    for kk in k:
      parts.append(b' '.join(words[i] for i in idx[at:at + kk]))
      at += kk
    off = np.zeros(n + 1, np.int64)
    np.cumsum([len(x) for x in parts], out=off[1:])
    return pa.Array.from_buffers(pa.string(), n, [None, pa.py_buffer(off.astype(np.int32)), pa.py_buffer(b''.join(parts))])

  return pa.Table.from_arrays([col(), col(), pa.array(rng.random(n) < 0.5), pa.array(rng.integers(0, 512, n).astype(np.uint16)),
                               pa.array(rng.integers(0, 8, n))], names=['A', 'B', 'is_random_next', 'num_tokens', 'bin_id'])


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--rows', type=int, default=300_000)
  ap.add_argument('--files', type=int, default=512)
  ap.add_argument('--threads', default='1,4,8,16')
  ap.add_argument('--dirs', default='/tmp,/dev/shm')
  ap.add_argument('--pinned', action='store_true',
                  help='the string buffers in pinned host memory (torch pin_memory), as the writer hands them over')
  a = ap.parse_args()
  tb = table(a.rows, 620)
  if a.pinned:
    import torch

    def pin(arr):
      bufs = arr.buffers()
      out = []
      for b in bufs:
        if b is None:
          out.append(None)
          continue
        h = torch.empty(b.size, dtype=torch.uint8, pin_memory=True)
        h.numpy()[:] = np.frombuffer(b, dtype=np.uint8)
        out.append(pa.py_buffer(h.numpy()))
      return pa.Array.from_buffers(arr.type, len(arr), out)

    tb = pa.Table.from_arrays([pin(c.combine_chunks()) for c in tb.columns], names=tb.column_names)
  per = a.rows // a.files
  dict_cols = ['is_random_next', 'num_tokens', 'bin_id']
  out = {'rows': a.rows, 'files': a.files, 'pinned': a.pinned, 'table_mb': tb.nbytes / 1e6, 'cpu_count': os.cpu_count(), 'runs': []}

  def go(k, sink):
    d = tempfile.mkdtemp(dir=sink) if sink else None
    def one(i):
      t = tb.slice(i * per, per)
      if d is None:
        s = pa.BufferOutputStream()
        pq.write_table(t, s, compression='snappy', use_dictionary=dict_cols)
        return s.getvalue().size
      p = os.path.join(d, 'part.%d.parquet' % i)
      pq.write_table(t, p, compression='snappy', use_dictionary=dict_cols)
      return os.path.getsize(p)
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(k) as ex:
      nb = sum(ex.map(one, range(a.files)))
    el = time.perf_counter() - t0
    if d:
      shutil.rmtree(d, ignore_errors=True)
    return el, nb

  go(1, None)  # warm pyarrow's lazy imports
  for sink in [None] + [x for x in a.dirs.split(',') if x and os.path.isdir(x)]:
    for k in [int(x) for x in a.threads.split(',')]:
      el = min(go(k, sink)[0] for _ in range(2))
      _, nb = go(k, sink)
      r = {'sink': sink or 'memory', 'threads': k, 'seconds': el, 'rows_per_s': a.rows / el, 'parquet_mb': nb / 1e6,
           'mb_per_s': nb / 1e6 / el}
      out['runs'].append(r)
      print(json.dumps(r), flush=True)
  print(json.dumps(out))


if __name__ == '__main__':
  main()
