"""Input layer of the preprocessor front end (reference: lddl/dask/readers.py).

The reference reads its sources with ``dask.bag.read_text`` (readers.py:60-70):
one record per LINE, stripped, empty ones dropped (``_filter_empty_strs``,
readers.py:31-32), then sampled.  Lines are what Python's text mode calls
lines:

* BERT sources (``linedelimiter=None``): universal newlines -- a line ends at
  ``\\n``, ``\\r\\n`` or ``\\r`` and nowhere else (``str.splitlines`` would also
  break on ``\\v \\f \\x1c-\\x1e \\x85 \\u2028 \\u2029``, which read_text never
  does);
* CodeBERT (``read_code``, readers.py:130-139): ``linedelimiter="\\r\\n"``, a
  line ends only at ``\\r\\n``.

Partitions: ``read_text(files, blocksize=B)`` gives every file the blocks of
``dask.bytes.read_bytes`` (``dask_blocks``: a file of S > 0 bytes gets
max(1, S // B) blocks); without a block size every file is one partition.
``--num-blocks`` turns into a block size via ``estimate_block_size``
(readers.py:48-57, over ALL files of the given source roots).  The CodeBERT
preprocessor ignores both flags: one partition per file
(pretrain_codebert.py:479-485).

``RecordIndex`` holds (file, byte offset, byte length) of every stripped,
non-empty record instead of the strings, so a rank keeps only integers for
the whole input and reads the text of its own partitions lazily (mmap).
"""
import mmap
import os

import numpy as np

__all__ = ['find_files_under', 'parse_str_of_num_bytes', 'estimate_block_size', 'dask_blocks', 'iter_lines',
           'RecordIndex', 'count_partitions']

# bytes for which str.isspace() holds among ASCII (\t \n \v \f \r \x1c-\x1f, space)
_ASCII_WS = np.zeros(256, dtype=bool)
_ASCII_WS[[9, 10, 11, 12, 13, 28, 29, 30, 31, 32]] = True


def find_files_under(path, extensions=('.txt',)):
  """readers.py:35-41: every file under path with one of the extensions, sorted"""
  out = []
  for d, _, names in os.walk(path):
    out.extend(os.path.join(d, n) for n in names if os.path.splitext(n)[1] in extensions)
  return sorted(out)


def parse_str_of_num_bytes(s, return_str=False):
  """lddl/download/utils.py:42-51, the --block-size type: n[KMG] (x 1024**k).

  Like the reference, the last character is always taken as the unit: a
  plain number loses its last digit ('1000' -> 100 bytes)."""
  try:
    power = 'kmg'.find(s[-1].lower()) + 1
    size = float(s[:-1]) * 1024**power
  except ValueError:
    raise ValueError('Invalid size: {}'.format(s))
  if return_str:
    return s
  return int(size)


def estimate_block_size(paths, num_blocks):
  """readers.py:48-57: round(total bytes of every file under the given roots
  (None skipped) / num_blocks)"""
  total = 0
  for p in paths:
    if p is None:
      continue
    total += sum(os.path.getsize(f) for f in find_files_under(p))
  return round(total / num_blocks)


def dask_blocks(size, blocksize):
  """Number of blocks dask.bytes.read_bytes cuts a file of `size` bytes into
  (the blocksize is shrunk to size / (size // blocksize) so the parts are
  even; an empty file has none)."""
  if size == 0:
    return 0
  if size % blocksize and size > blocksize:
    bs1 = size / (size // blocksize)
  else:
    bs1 = blocksize
  place, n = 0, 1
  while size - place > (bs1 * 2) - 1:
    place += bs1
    n += 1
  return n


def count_partitions(files, blocksize=None):
  """Partitions of read_text(files, blocksize): one per file without a block
  size, else the read_bytes blocks of every file."""
  if blocksize is None:
    return len(files)
  return sum(dask_blocks(os.path.getsize(f), blocksize) for f in files)


def iter_lines(path, linedelimiter=None):
  """The stripped, non-empty records of one file, as read_text + strip +
  filter yield them (a reference-semantics restatement on Python's own text
  mode, used by tests and small inputs)."""
  newline = None if linedelimiter is None else linedelimiter
  with open(path, encoding='utf-8', newline=newline) as f:
    for line in f:
      s = line.strip()
      if s:
        yield s


def _line_spans(buf, crlf_only):
  """(start, end) byte spans of the lines of buf (terminators excluded)"""
  n = len(buf)
  if n == 0:
    return np.zeros(0, np.int64), np.zeros(0, np.int64)
  lf = np.flatnonzero(buf == 10)
  if crlf_only:
    t = lf[lf > 0]
    t = t[buf[t - 1] == 13] - 1  # the CR of each CR LF pair
    tl = np.full(len(t), 2, np.int64)
  else:
    # universal newlines: CR LF, lone CR and lone LF each end a line (one
    # pass for each terminator byte; CRs are rare in practice)
    cr = np.flatnonzero(buf == 13)
    if len(cr):
      lone_lf = lf[~np.isin(lf - 1, cr)]
      t = np.sort(np.concatenate([cr, lone_lf]))
      tl = np.ones(len(t), np.int64)
      nxt = np.minimum(t + 1, n - 1)
      tl[(buf[t] == 13) & (buf[nxt] == 10) & (t + 1 < n)] = 2
    else:
      t = lf
      tl = np.ones(len(t), np.int64)
  starts = np.concatenate([[0], t + tl]).astype(np.int64)
  ends = np.concatenate([t, [n]]).astype(np.int64)
  if starts[-1] >= n:  # the text ends with a terminator: no final line
    starts, ends = starts[:-1], ends[:-1]
  return starts, ends


def _strip_spans(buf, starts, ends):
  """str.strip() on each line span, in bytes; returns (offsets, lengths) of
  the non-empty ones.  ASCII whitespace vectorised; a line whose first or
  last non-ASCII-space byte is non-ASCII is decoded to strip Unicode spaces."""
  if len(starts) == 0:
    return np.zeros(0, np.int64), np.zeros(0, np.int64)
  # ASCII whitespace at the span edges, peeled one byte per round over the
  # spans that still have some (almost none: no pass over every byte)
  s, e = starts.astype(np.int64).copy(), ends.astype(np.int64).copy()
  act = np.flatnonzero(s < e)
  while len(act):
    act = act[_ASCII_WS[buf[s[act]]]]
    s[act] += 1
    act = act[s[act] < e[act]]
  act = np.flatnonzero(s < e)
  while len(act):
    act = act[_ASCII_WS[buf[e[act] - 1]]]
    e[act] -= 1
    act = act[s[act] < e[act]]
  keep = s < e
  off, ln = s[keep], (e - s)[keep]
  if len(off):
    # a line may start or end with a Unicode space (str.isspace beyond ASCII:
    # U+0085, U+00A0 lead 0xC2; U+1680, U+2000-U+205F, U+3000 lead 0xE1-0xE3)
    # only if its first byte or its last character's lead byte is one of
    # those: only such lines are decoded (not every CJK line)
    end = off + ln
    f0 = buf[off]
    l2 = np.where(ln >= 2, buf[np.maximum(end - 2, off)], 0)
    l3 = np.where(ln >= 3, buf[np.maximum(end - 3, off)], 0)
    hi = ((f0 == 0xC2) | ((f0 >= 0xE1) & (f0 <= 0xE3)) | (l2 == 0xC2) | ((l3 >= 0xE1) & (l3 <= 0xE3)))
    for k in np.flatnonzero(hi):
      raw = bytes(buf[off[k]:off[k] + ln[k]])
      t = raw.decode('utf-8')
      lead = len(t) - len(t.lstrip())
      core = t.strip()
      a = len(t[:lead].encode('utf-8'))
      off[k], ln[k] = off[k] + a, len(core.encode('utf-8'))
    nonempty = ln > 0
    off, ln = off[nonempty], ln[nonempty]
  return off, ln


INDEX_WINDOW = 64 << 20  # bytes of a file indexed at a time


class RecordIndex:
  """(file, offset, length) of every record of the given files, in file order
  then line order -- the order of read_text's bag before sampling."""

  def __init__(self, files, fid, off, ln):
    self.files = list(files)
    self.fid = np.asarray(fid, np.int32)
    self.off = np.asarray(off, np.int64)
    self.len = np.asarray(ln, np.int64)
    self._mm = {}

  def __len__(self):
    return len(self.off)

  @staticmethod
  def index_file(path, linedelimiter=None):
    """offsets / lengths of the records of one file"""
    if linedelimiter not in (None, '\r\n'):
      raise ValueError('linedelimiter must be None (universal newlines) or "\\r\\n"')
    size = os.path.getsize(path)
    if size == 0:
      return np.zeros(0, np.int64), np.zeros(0, np.int64)
    buf = np.memmap(path, dtype=np.uint8, mode='r')
    # the whole file in one C pass when the host library is there (the same
    # spans; LDDL_SPLIT_NATIVE=0 keeps the numpy windows below)
    if os.environ.get('LDDL_SPLIT_NATIVE', '1') != '0':
      from . import splitnative
      got = splitnative.line_spans(buf, linedelimiter == '\r\n')
      if got is not None:
        return _strip_spans(buf, *got)
    # windows of ~INDEX_WINDOW bytes, each cut right after a line feed (a
    # window starts a line; a \r\n pair never splits), so the per-byte masks
    # and indices live for one window at a time, not the whole file
    crlf = linedelimiter == '\r\n'

    def cuts(lo, hi):  # line feeds in [lo, hi) that end a line (\r\n only: after a \r)
      w = buf[lo:hi]
      lf = np.flatnonzero(w == 10)
      if crlf and len(lf):
        prev = np.where(lf > 0, w[np.maximum(lf - 1, 0)], buf[lo - 1] if lo > 0 else 0)
        lf = lf[prev == 13]
      return lf + lo

    offs, lns = [], []
    a = 0
    while a < size:
      b = min(size, a + INDEX_WINDOW)
      if b < size:
        lf = cuts(a, b)
        while len(lf) == 0 and b < size:  # a line longer than the window
          b2 = min(size, b + INDEX_WINDOW)
          lf = cuts(b, b2)
          b = b2
        if len(lf):
          b = int(lf[-1]) + 1
      w = buf[a:b]
      s, e = _line_spans(w, linedelimiter == '\r\n')
      o, l = _strip_spans(w, s, e)
      offs.append(o + a)
      lns.append(l)
      a = b
    return np.concatenate(offs), np.concatenate(lns)

  @classmethod
  def build(cls, files, linedelimiter=None, file_ids=None):
    """Index the files (or only those of file_ids, for a rank's share)."""
    fids, offs, lns = [], [], []
    for i, f in enumerate(files):
      if file_ids is not None and i not in file_ids:
        continue
      o, l = cls.index_file(f, linedelimiter)
      fids.append(np.full(len(o), i, np.int32))
      offs.append(o)
      lns.append(l)
    cat = lambda a, t: np.concatenate(a).astype(t) if a else np.zeros(0, t)
    return cls(files, cat(fids, np.int32), cat(offs, np.int64), cat(lns, np.int64))

  @classmethod
  def merge(cls, files, parts):
    """Per-rank indexes of disjoint file subsets -> one index in file order."""
    fid = np.concatenate([p.fid for p in parts]) if parts else np.zeros(0, np.int32)
    off = np.concatenate([p.off for p in parts]) if parts else np.zeros(0, np.int64)
    ln = np.concatenate([p.len for p in parts]) if parts else np.zeros(0, np.int64)
    order = np.lexsort((off, fid))
    return cls(files, fid[order], off[order], ln[order])

  def text(self, i):
    """record i as str (strict UTF-8, as read_text decodes)"""
    f = int(self.fid[i])
    mm = self._mm.get(f)
    if mm is None:
      with open(self.files[f], 'rb') as fh:
        mm = self._mm[f] = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ)
    o = int(self.off[i])
    return mm[o:o + int(self.len[i])].decode('utf-8')

  def texts(self, idx):
    return [self.text(int(i)) for i in idx]

  def raw(self, i):
    """record i's bytes (not decoded: the native splitter validates them)"""
    f = int(self.fid[i])
    mm = self._mm.get(f)
    if mm is None:
      with open(self.files[f], 'rb') as fh:
        mm = self._mm[f] = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ)
    o = int(self.off[i])
    return mm[o:o + int(self.len[i])]

  def raws(self, idx):
    return [self.raw(int(i)) for i in idx]

  def close(self):
    for mm in self._mm.values():
      mm.close()
    self._mm = {}

  def __getstate__(self):  # picklable (no open maps)
    d = dict(self.__dict__)
    d['_mm'] = {}
    return d
