"""ORACLE -- test infrastructure only (tests/, __graft_entry__.smoke(),
bench.py cpu_baseline).  Never imported by lddl_amd/.

ctypes wrapper of oracle/liboracle.so (C restatement of the HF tokenizers
pipeline, see tokenizer_oracle.c) plus the Python restatement of the packer
(oracle/pack_oracle.py).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
TABLE = os.path.join(ROOT, 'lddl_amd', 'data', 'unicode_table.bin')

_L = None


def lib():
  global _L
  if _L is None:
    p = os.path.join(HERE, 'liboracle.so')
    if not os.path.exists(p):
      import subprocess
      subprocess.run(['make', '-s'], cwd=HERE, check=True)
    L = ctypes.CDLL(p)
    L.orc_tok_create.restype = ctypes.c_void_p
    L.orc_tok_create.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    L.orc_tok_destroy.argtypes = [ctypes.c_void_p]
    L.orc_tok_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                              ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.orc_words.restype = ctypes.c_int64
    L.orc_words.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_int64]
    L.orc_tok_vocab_size.argtypes = [ctypes.c_void_p]
    L.orc_tok_special_id.argtypes = [ctypes.c_void_p, ctypes.c_int]
    _L = L
  return _L


class OracleTokenizer:
  def __init__(self, vocab_file):
    self.h = lib().orc_tok_create(vocab_file.encode(), TABLE.encode())
    if not self.h:
      raise RuntimeError('oracle tokenizer: cannot load %s' % vocab_file)

  def __del__(self):
    if getattr(self, 'h', None):
      lib().orc_tok_destroy(self.h)
      self.h = None

  def run(self, data, sent_off, max_tok=512, nthreads=1, out=None):
    """Sparse output like the HIP path: (ids int32[nbytes], ntok int32[n_sent]).
    out: preallocated (ids, ntok) of at least those sizes (a timing caller
    touches them first, so page faults stay out of the timed call)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    sent_off = np.ascontiguousarray(sent_off, dtype=np.int64)
    n = len(sent_off) - 1
    if out is None:
      ids = np.zeros(max(1, int(sent_off[-1] - sent_off[0])), dtype=np.int32)
      ntok = np.zeros(max(1, n), dtype=np.int32)
    else:
      ids, ntok = out
      assert ids.dtype == np.int32 and ntok.dtype == np.int32 and ids.flags.c_contiguous
      assert len(ids) >= int(sent_off[-1] - sent_off[0]) and len(ntok) >= n
    lib().orc_tok_run(self.h, data.ctypes.data, sent_off.ctypes.data, n, max_tok, ids.ctypes.data,
                      ntok.ctypes.data, nthreads)
    return ids, ntok[:n]

  def words(self, s):
    b = s.encode('utf-8')
    buf = ctypes.create_string_buffer(len(b) * 12 + 64)
    n = lib().orc_words(self.h, b, len(b), buf, len(buf))
    if n < 0:
      raise RuntimeError('orc_words overflow')
    return buf.raw[:n].decode('utf-8').split('\n')[:-1]


def compact(ids, ntok, sent_off):
  """sparse (ids by byte offset) -> list of per-sentence id lists"""
  base = sent_off[0]
  return [ids[sent_off[i] - base:sent_off[i] - base + ntok[i]] for i in range(len(ntok))]
