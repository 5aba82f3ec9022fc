"""Parquet encode worker (writer.ProcessEncoder): runs in a pool of host
processes, so the per-file Python work of pyarrow's writer (the part that
holds the GIL: writer construction, schema, file open / close) runs in
parallel instead of serialising a thread pool on small files.

A batch's columns arrive in a shared slot file under /dev/shm (mapped here
once per slot generation): string / binary columns as int64 offsets + bytes,
fixed-width columns as raw values.  Each task writes a run of the batch's
files, each a row range, zero-copy from the mapping.  Imports only numpy and
pyarrow (no torch, no GPU).
"""
import mmap
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

_MAPS = {}  # slot path -> (mmap, size)

_FIXED = {'bool': np.bool_, 'u16': np.uint16, 'i64': np.int64}
_ARROW = {'u16': pa.uint16(), 'i64': pa.int64()}


def _map(path, size):
  m = _MAPS.get(path)
  if m is None or m[1] < size:
    if m is not None:
      try:
        m[0].close()
      except BufferError:  # (a view still alive: leave it to the collector)
        pass
    fd = os.open(path, os.O_RDONLY)
    try:
      mm = mmap.mmap(fd, size, prot=mmap.PROT_READ)
    finally:
      os.close(fd)
    m = (mm, size)
    _MAPS[path] = m
  return m[0]


def _var_column(typ, mm, off_pos, n, data_pos, lo, hi):
  """rows [lo, hi) of an (int64 offsets from 0, bytes) column, offsets
  rebased to the file's first row"""
  off = np.frombuffer(mm, dtype=np.int64, count=n + 1, offset=off_pos)
  o = off[lo:hi + 1] - off[lo]
  nb = int(o[-1])
  data = pa.py_buffer(memoryview(mm)[data_pos + int(off[lo]):data_pos + int(off[lo]) + nb])
  if nb < 2**31:
    return pa.Array.from_buffers(typ, hi - lo, [None, pa.py_buffer(o.astype(np.int32)), data])
  big = pa.large_string() if typ == pa.string() else pa.large_binary()
  return pa.Array.from_buffers(big, hi - lo, [None, pa.py_buffer(np.ascontiguousarray(o)), data]).cast(typ)


def _fixed_column(kind, mm, pos, n, lo, hi):
  x = np.frombuffer(mm, dtype=_FIXED[kind], count=n, offset=pos)[lo:hi]
  if kind == 'bool':
    return pa.Array.from_buffers(pa.bool_(), hi - lo, [None, pa.py_buffer(np.packbits(x, bitorder='little'))])
  return pa.Array.from_buffers(_ARROW[kind], hi - lo, [None, pa.py_buffer(np.ascontiguousarray(x))])


def encode(slot, size, n, cols, schema, files, compression, dict_cols):
  """cols: (name, kind, pos, data_pos) per schema column in order; kind
  'str' / 'bin' (offsets at pos, bytes at data_pos) or 'bool' / 'u16' / 'i64';
  files: (path, lo, hi) row ranges of the batch.  Returns the bytes written."""
  mm = _map(slot, size)
  total = 0
  for path, lo, hi in files:
    arrs = []
    for name, kind, pos, dpos in cols:
      if kind in ('str', 'bin'):
        arrs.append(_var_column(pa.string() if kind == 'str' else pa.binary(), mm, pos, n, dpos, lo, hi))
      else:
        arrs.append(_fixed_column(kind, mm, pos, n, lo, hi))
    t = pa.Table.from_arrays(arrs, schema=schema)
    pq.write_table(t, path, compression=compression, use_dictionary=dict_cols)
    del t, arrs
    total += os.path.getsize(path)
  return total
