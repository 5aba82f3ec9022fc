"""Host side of the parquet writer (no GPU): the masked_lm_positions bytes
equal lddl/utils.py:98-102 serialize_np_array, schemas match
pretrain.py:450-471 / pretrain_codebert.py:499-510."""
import io
import os

import numpy as np
import pyarrow as pa

from lddl_amd import writer


def _serialize(a):
  b = io.BytesIO()
  np.save(b, a)
  return b.getvalue()


def test_npy_positions_match_np_save():
  rng = np.random.default_rng(0)
  k = rng.integers(0, 160, 300)
  k[:3] = 0
  off = np.zeros(len(k) + 1, dtype=np.int64)
  np.cumsum(k, out=off[1:])
  pos = rng.integers(0, 1024, int(off[-1])).astype(np.uint16)
  o, d = writer.npy_positions(off, pos)
  for r in range(len(k)):
    assert d[o[r]:o[r + 1]].tobytes() == _serialize(pos[off[r]:off[r + 1]].astype(np.uint16))
  col = writer._arrow(pa.binary(), o, d, 10, 20)
  assert col.to_pylist() == [_serialize(pos[off[r]:off[r + 1]]) for r in range(10, 20)]


def test_npy_positions_empty():
  o, d = writer.npy_positions(np.zeros(1, np.int64), np.zeros(0, np.uint16))
  assert o.tolist() == [0] and len(d) == 0


def test_schemas():
  assert writer.schema().names == ['A', 'B', 'is_random_next', 'num_tokens']
  assert writer.schema(masking=True, binned=True).names == [
      'A', 'B', 'is_random_next', 'num_tokens', 'masked_lm_positions', 'masked_lm_labels', 'bin_id']
  s = writer.schema(codebert=True, binned=True)
  assert s.names == ['id', 'doc', 'code', 'num_tokens', 'bin_id']
  assert s.field('num_tokens').type == pa.uint16() and s.field('bin_id').type == pa.int64()


def test_arrow_slices_and_large_offsets():
  data = np.frombuffer(b'abcdefghij', dtype=np.uint8)
  off = np.array([0, 2, 2, 5, 10], dtype=np.int64)
  assert writer._arrow(pa.string(), off, data, 1, 4).to_pylist() == ['', 'cde', 'fghij']
  assert writer._arrow(pa.string(), off, data, 2, 2).to_pylist() == []


def test_process_encoder_writes_what_pyarrow_writes(tmp_path):
  """writer.ProcessEncoder (forked workers, the batch's columns in a shared
  slot file) writes files with the same tables as pq.write_table of the same
  row ranges, for every column kind, across slot reuse and growth"""
  import pyarrow.parquet as pq
  rng = np.random.default_rng(5)
  enc = writer.ProcessEncoder(workers=2, slots=2)
  try:
    sch = writer.schema(masking=True, binned=True)
    for batch, n in enumerate((50, 3000, 0, 700)):
      def var(binary=False):
        lens = rng.integers(0, 40, size=n)
        off = np.zeros(n + 1, np.int64)
        np.cumsum(lens, out=off[1:])
        data = rng.integers(97, 123, size=int(off[-1])).astype(np.uint8)
        return off, data
      cols = {nm: var() for nm in ('A', 'B', 'masked_lm_positions', 'masked_lm_labels')}
      fixed = {'is_random_next': ('bool', rng.random(n) < 0.5), 'num_tokens': ('u16', rng.integers(0, 600, n).astype(np.uint16)),
               'bin_id': ('i64', rng.integers(0, 8, n).astype(np.int64))}
      specs = [(nm, 'bin' if nm == 'masked_lm_positions' else 'str') + cols[nm] if nm in cols else
               (nm, fixed[nm][0], fixed[nm][1], None) for nm in sch.names]
      cuts = np.unique(np.concatenate([[0, n], rng.integers(0, n + 1, size=7)]))
      files = [(str(tmp_path / ('b%d_f%d.parquet' % (batch, i))), int(a), int(b))
               for i, (a, b) in enumerate(zip(cuts[:-1], cuts[1:]))]
      futs = enc.submit_batch(n, specs, sch, files, 'snappy', ['is_random_next', 'num_tokens', 'bin_id'])
      for f_ in futs:
        f_.result()
      for path, lo, hi in files:
        got = pq.read_table(path)
        arrs = []
        for nm, fd in zip(sch.names, sch):
          if nm in cols:
            off, data = cols[nm]
            arrs.append(writer._arrow(fd.type, off, data, lo, hi))
          else:
            arrs.append(writer.np_array(fixed[nm][1][lo:hi]))
        exp = pa.Table.from_arrays(arrs, schema=sch)
        assert got.equals(exp), (batch, path)
  finally:
    enc.close()
  assert not os.path.exists(enc.dir)


def test_process_encoder_slot_moves_to_disk_when_tmpfs_is_full(tmp_path, monkeypatch):
  """a slot that grows past the tmpfs' free space reserves it
  (posix_fallocate) and so sees ENOSPC as an OSError, and moves to a
  directory on disk instead of faulting (SIGBUS) in the copy"""
  import errno
  import pyarrow.parquet as pq
  enc = writer.ProcessEncoder(workers=1, slots=1)
  real = os.posix_fallocate
  full = enc.dir

  def falloc(fd, off, n):
    if os.readlink('/proc/self/fd/%d' % fd).startswith(full):
      raise OSError(errno.ENOSPC, 'No space left on device')
    return real(fd, off, n)
  monkeypatch.setattr(os, 'posix_fallocate', falloc)
  try:
    sch = writer.schema()
    n = 300
    off = np.arange(n + 1, dtype=np.int64) * 3
    data = np.frombuffer(b'abc' * n, dtype=np.uint8)
    specs = [('A', 'str', off, data), ('B', 'str', off, data), ('is_random_next', 'bool', np.zeros(n, bool), None),
             ('num_tokens', 'u16', np.full(n, 7, np.uint16), None)]
    f = str(tmp_path / 'x.parquet')
    for f_ in enc.submit_batch(n, specs, sch, [(f, 0, n)], 'snappy', ['is_random_next', 'num_tokens']):
      f_.result()
    assert enc.disk_dir is not None and enc.slots[0]['path'].startswith(enc.disk_dir)
    t = pq.read_table(f)
    assert t.column('A').to_pylist() == ['abc'] * n and t.column('num_tokens').to_pylist() == [7] * n
  finally:
    enc.close()
  assert not os.path.exists(enc.dir) and not os.path.exists(enc.disk_dir)


def test_host_var_all_empty_strings():
  """Arrow may leave the data buffer out of a slice whose strings
  are all empty"""
  a = pa.array(['', '', ''], pa.string())
  off, data = writer._host_var(a, 0, 3)
  assert off.tolist() == [0, 0, 0, 0] and data.size == 0
  b = pa.array(['x', '', '', 'yz'], pa.string())
  off, data = writer._host_var(b, 1, 2)
  assert off.tolist() == [0, 0, 0] and data.size == 0
  off, data = writer._host_var(b, 2, 2)
  assert off.tolist() == [0, 0, 2] and bytes(data) == b'yz'
