"""Host side of the parquet writer (no GPU): the masked_lm_positions bytes
equal lddl/utils.py:98-102 serialize_np_array, schemas match
pretrain.py:450-471 / pretrain_codebert.py:499-510."""
import io

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
