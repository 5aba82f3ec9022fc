"""The CLI's sentence split in C (lddl_amd/host/split_rules.c, libsplit.so):
split_id_text + the rule-based splitter + split_records' strip / drop, over
the records' raw UTF-8 bytes, with the exact result of the Python path
(preprocess.split_records with preprocess._rule_split).  BERT records only;
CodeBERT records and NLTK Punkt stay in Python.  The code point properties
the rules read come from this Python's unicodedata (one table, built once
per process or loaded from the cache next to the library)."""
import ctypes
import os
import unicodedata

import numpy as np

from . import synth

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, 'libsplit.so')
P_SPACE, P_UPPER, P_DIGIT, P_ALPHA1 = 1, 2, 4, 8
_STATE = {}


def props_table():
  """uint8 per code point: str.isspace / isupper / isdigit / one-letter
  lowercase alphabetic, for this interpreter's Unicode version"""
  t = _STATE.get('tab')
  if t is not None:
    return t
  cache = os.path.join(_PKG, 'data', 'split_props_%s.bin' % unicodedata.unidata_version)
  if os.path.exists(cache) and os.path.getsize(cache) == 0x110000:
    t = np.fromfile(cache, dtype=np.uint8)
  else:
    t = np.zeros(0x110000, dtype=np.uint8)
    for c in range(0x110000):
      ch = chr(c)
      f = 0
      if ch.isspace():
        f |= P_SPACE
      if ch.isupper():
        f |= P_UPPER
      if ch.isdigit():
        f |= P_DIGIT
      lo = ch.lower()
      if len(lo) == 1 and lo.isalpha():
        f |= P_ALPHA1
      t[c] = f
    try:
      t.tofile(cache + '.tmp%d' % os.getpid())
      os.replace(cache + '.tmp%d' % os.getpid(), cache)
    except OSError:
      pass
  _STATE['tab'] = t
  return t


def _lib():
  L = _STATE.get('lib')
  if L is None:
    if not os.path.exists(LIB_PATH):
      return None
    L = ctypes.CDLL(LIB_PATH)
    f = L.lddl_split_rules
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                  ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]
    g = L.lddl_line_spans
    g.restype = ctypes.c_int64
    g.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    _STATE['lib'] = L
  return L


def available():
  return _lib() is not None


def _p(a):
  return ctypes.c_void_p(a.ctypes.data)


def split_raw(raws):
  """BERT records as bytes -> (synth.Corpus, doc ids) exactly as
  preprocess.split_records([r.decode() for r in raws], False, _rule_split);
  None when the library is absent or a record is not valid UTF-8 (the
  Python path then decodes it and raises as before)."""
  L = _lib()
  if L is None:
    return None
  tab = props_table()
  n = len(raws)
  lens = np.fromiter((len(r) for r in raws), dtype=np.int64, count=n)
  rec_off = np.zeros(n + 1, dtype=np.int64)
  np.cumsum(lens, out=rec_off[1:])
  joined = b''.join(raws)
  buf = np.frombuffer(joined, dtype=np.uint8) if n else np.zeros(1, np.uint8)
  total = int(rec_off[-1])
  out = np.empty(max(total, 1), dtype=np.uint8)
  doc = np.zeros(n + 1, dtype=np.int64)
  ids = np.zeros(2 * max(n, 1), dtype=np.int64)
  bad = ctypes.c_int64(-1)
  cap = total // 32 + n + 64
  while True:
    soff = np.zeros(cap + 1, dtype=np.int64)
    ns = L.lddl_split_rules(_p(buf), _p(rec_off), n, _p(tab), _p(out), out.size, _p(soff), cap, _p(doc), _p(ids),
                            ctypes.byref(bad))
    if ns == -3 and cap <= total:  # (non-empty sentences: at most one per byte)
      cap = min(cap * 4, total + 1)
      continue
    if ns < 0:
      return None
    break
  corpus = synth.Corpus(out[:int(soff[ns])], soff[:ns + 1], doc, None)
  idl = ids.tolist()
  doc_ids = [joined[idl[2 * r]:idl[2 * r + 1]].decode('utf-8') for r in range(n)]
  return corpus, doc_ids


def _spans_piece(L, base, lo, hi, crlf_only):
  """the line spans of buf[lo, hi) (base = the buffer's address), offsets
  relative to lo"""
  n = hi - lo
  if n <= 0:
    return np.zeros(0, np.int64), np.zeros(0, np.int64)
  p = ctypes.c_void_p(base + lo)
  cap = n // 32 + 1024  # (one call for lines of >= 32 B on average; else count, then fill)
  s, e = np.empty(cap, np.int64), np.empty(cap, np.int64)
  m = L.lddl_line_spans(p, n, 1 if crlf_only else 0, _p(s), _p(e), cap)
  if m > cap:
    s, e = np.empty(m, np.int64), np.empty(m, np.int64)
    L.lddl_line_spans(p, n, 1 if crlf_only else 0, _p(s), _p(e), m)
  return s[:m], e[:m]


def _cut_after_terminator(buf, b, crlf_only):
  """the first position after a line terminator at or past b (a piece may
  start there: no CR LF pair straddles it), or len(buf)"""
  n, w = len(buf), 1 << 16
  pat = b'\r\n' if crlf_only else b'\n'
  lo = max(b - 1, 0) if crlf_only else b
  while lo < n:
    hi = min(n, lo + w)
    k = bytes(buf[lo:hi]).find(pat)
    if k >= 0:
      return lo + k + len(pat)
    lo = hi - (len(pat) - 1)
    if hi == n:
      break
    w *= 4
  return n


def line_spans(buf, crlf_only, threads=None, min_piece=64 << 20):
  """readers._line_spans in C (memchr): (starts, ends) int64, or None
  without the library.  A large buffer is cut after line terminators into
  pieces indexed on threads (ctypes releases the GIL): a file read through
  a memory map spends most of a single pass in first-touch page faults."""
  L = _lib()
  if L is None:
    return None
  n = len(buf)
  if n == 0:
    return np.zeros(0, np.int64), np.zeros(0, np.int64)
  base = buf.ctypes.data
  if threads is None:
    from .hostinfo import cpu_share
    threads = cpu_share()
  k = max(1, min(int(threads), n // max(1, min_piece)))
  if k == 1:
    return _spans_piece(L, base, 0, n, crlf_only)
  cuts = [0]
  for i in range(1, k):
    c = _cut_after_terminator(buf, max(i * n // k, cuts[-1]), crlf_only)
    if cuts[-1] < c < n:
      cuts.append(c)
  cuts.append(n)
  from concurrent.futures import ThreadPoolExecutor
  with ThreadPoolExecutor(len(cuts) - 1) as ex:
    parts = list(ex.map(lambda i: _spans_piece(L, base, cuts[i], cuts[i + 1], crlf_only), range(len(cuts) - 1)))
  return (np.concatenate([s + cuts[i] for i, (s, _) in enumerate(parts)]),
          np.concatenate([e + cuts[i] for i, (_, e) in enumerate(parts)]))
