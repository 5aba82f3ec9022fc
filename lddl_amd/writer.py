"""Parquet shards in the reference's schema, from GPU-rendered string columns.

The reference turns every packed instance into a dict of strings
(pretrain.py:348-360, pretrain_codebert.py:425-432) and writes them with
``to_parquet`` (unbinned: ``part.{i}.parquet``, pretrain.py:472-478) or
``to_parquet_binned`` (one file per bin, ``part.{i}.parquet_{b}``, every bin
written even when empty, binning.py:353-431):

  BERT      A string, B string, is_random_next bool, num_tokens uint16
            [, masked_lm_positions binary (np.save bytes of uint16[k],
               lddl/utils.py:98-102), masked_lm_labels string]
            [, bin_id int64]                               pretrain.py:450-498
  CodeBERT  id string, doc string, code string, num_tokens uint16
            [, bin_id int64]                       pretrain_codebert.py:495-537

Here the rows of a pack call are already in file order on the device
(partition-major, bin-major, shuffled order within a bin), so a file is a
contiguous row range.  The string columns are rendered on the GPU by
``lddl_render_strings`` (Arrow layout: offsets + UTF-8 bytes) in row batches,
copied to the host once and wrapped zero-copy into Arrow arrays; the host only
slices offsets per file and runs the parquet encoder.
"""
import concurrent.futures
import ctypes
import io
import os
import time

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import torch

from . import _lib
from .tokenizer import _ptr, _stream

SEG0, SEG1, ROW, SPAN = 0, 1, 2, 3
from .hostinfo import DENSE_COLS  # noqa: E402  (re-exported: writer.DENSE_COLS)

BERT_SCHEMA = [('A', pa.string()), ('B', pa.string()), ('is_random_next', pa.bool_()),
               ('num_tokens', pa.uint16())]
MLM_SCHEMA = [('masked_lm_positions', pa.binary()), ('masked_lm_labels', pa.string())]
CODEBERT_SCHEMA = [('id', pa.string()), ('doc', pa.string()), ('code', pa.string()), ('num_tokens', pa.uint16())]


def schema(codebert=False, masking=False, binned=False):
  f = list(CODEBERT_SCHEMA if codebert else BERT_SCHEMA)
  if masking and not codebert:
    f += MLM_SCHEMA
  if binned:
    f.append(('bin_id', pa.int64()))
  return pa.schema(f)


def _host(t, stream=None):
  """device tensor -> numpy on the host through pinned memory (torch's
  caching host allocator: the block returns to the cache when the last view
  of it -- the Arrow buffers of the files still encoding -- is gone);
  synchronises the stream"""
  h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
  s = stream or torch.cuda.current_stream()
  with torch.cuda.stream(s):  # (the copy on the stream the render ran on)
    h.copy_(t, non_blocking=True)
  s.synchronize()
  return h.numpy()


def render(packer, tokens, row_off, row0, n_rows, segment, len0=None, len1=None, flags=None, codebert=False,
           stream=None, host=True):
  """One string column of rows [row0, row0 + n_rows) on the GPU.

  Returns (offsets int64[n_rows + 1] starting at 0, bytes uint8) on the host.
  """
  L = _lib.lib()
  dev = packer.device
  off = torch.empty(n_rows + 1, dtype=torch.int64, device=dev)
  nb = ctypes.c_int64(0)
  s = _stream(stream)
  args = (packer.tok.handle, _ptr(tokens), _ptr(row_off), _ptr(len0), _ptr(len1), _ptr(flags), row0, n_rows,
          segment, 1 if codebert else 0, _ptr(off))
  _lib.check(L.lddl_render_strings(*args, None, 0, ctypes.byref(nb), s))
  data = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=dev)
  _lib.check(L.lddl_render_strings(*args, _ptr(data), nb.value, ctypes.byref(nb), s))
  if not host:  # (device tensors: the process encoder copies them into its shared slot)
    return off, data[:nb.value]
  return _host(off, stream), _host(data[:nb.value], stream)


def render_masked(packer, res, row0, n_rows, segment, stream=None, host=True):
  """A (segment 0) / B (1) of span rows with the static masking applied
  (lddl_render_masked): (offsets, bytes) on the host as render()"""
  L = _lib.lib()
  off = torch.empty(n_rows + 1, dtype=torch.int64, device=packer.device)
  nb = ctypes.c_int64(0)
  s = _stream(stream)
  src, ln = (res.src0, res.len0) if segment == 0 else (res.src1, res.len1)
  args = (packer.tok.handle, _ptr(res.ids), _ptr(src), _ptr(ln), _ptr(res.len0), segment, _ptr(res.mlm_off),
          _ptr(res.mlm_pos), _ptr(res.mlm_token), row0, n_rows, _ptr(off))
  _lib.check(L.lddl_render_masked(*args, None, 0, ctypes.byref(nb), s))
  data = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=packer.device)
  _lib.check(L.lddl_render_masked(*args, _ptr(data), nb.value, ctypes.byref(nb), s))
  if not host:
    return off, data[:nb.value]
  return _host(off, stream), _host(data[:nb.value], stream)


def seg_columns(packer, res, r0, n, codebert=False, stream=None, host=True):
  """the two segment string columns (A / B, or doc / code) of rows
  [r0, r0 + n): rendered from the spans over the dense ids (res.spans) or
  from the materialised rows"""
  if res.spans and res.mlm_token is not None:
    return (render_masked(packer, res, r0, n, 0, stream, host), render_masked(packer, res, r0, n, 1, stream, host))
  if res.spans:
    return (render(packer, res.ids, res.src0, r0, n, SPAN, len0=res.len0, stream=stream, host=host),
            render(packer, res.ids, res.src1, r0, n, SPAN, len0=res.len1, stream=stream, host=host))
  kw = dict(len0=res.len0, len1=res.len1, flags=res.flags, codebert=codebert, stream=stream, host=host)
  return (render(packer, res.tokens, res.tok_off, r0, n, SEG0, **kw),
          render(packer, res.tokens, res.tok_off, r0, n, SEG1, **kw))


def row_docs(packer, res, n_copy=None, stream=None):
  """document index of every row of the pack result `res` (lddl_row_docs
  over res.pack, all rows on the device); the first n_copy of them copied to
  the host"""
  n_rows = res.n_pairs
  out = torch.empty(max(n_rows, 1), dtype=torch.int64, device=packer.device)
  _lib.check(_lib.lib().lddl_row_docs(packer.tok.handle, res.pack.handle, _ptr(out), _stream(stream)))
  return out[:n_rows if n_copy is None else min(n_copy, n_rows)].cpu().numpy()


_NPY_HDR = {}  # device -> (uint16 tensor [(kmax + 1) * H / 2], H bytes, kmax)


def npy_header_table(device, kmax=1024):
  """np.save's header of a uint16[k] array for every k <= kmax, back to
  back on the device (what lddl_render_npy prepends to each row), or None
  when the headers differ in length (then the host path builds the column)"""
  t = _NPY_HDR.get(device)
  if t is None or t[2] < kmax:
    hdr = [_npy_header(k) for k in range(kmax + 1)]
    if len({len(h) for h in hdr}) != 1 or len(hdr[0]) % 2:
      return None
    flat = np.concatenate(hdr).view(np.uint16)
    t = (torch.from_numpy(flat.view(np.int16).copy()).to(device), len(hdr[0]), kmax)
    _NPY_HDR[device] = t
  return t


def render_npy(packer, res, row0, n_rows, stream=None, host=True):
  """masked_lm_positions of rows [row0, row0 + n_rows) as np.save bytes
  per row on the GPU (lddl_render_npy): (offsets, bytes) on the host as
  render(), or None when the header table does not apply"""
  if os.environ.get('LDDL_NPY_HOST'):  # (A/B: the host path)
    return None
  kmax = 1024
  t = npy_header_table(packer.device, kmax)
  if t is None:
    return None
  hdr, hlen, kmax = t
  L = _lib.lib()
  off = torch.empty(n_rows + 1, dtype=torch.int64, device=packer.device)
  nb = ctypes.c_int64(0)
  s = _stream(stream)
  args = (packer.tok.handle, _ptr(res.mlm_off), _ptr(res.mlm_pos), row0, n_rows, _ptr(hdr), hlen, kmax, _ptr(off))
  _lib.check(L.lddl_render_npy(*args, None, 0, ctypes.byref(nb), s))
  data = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=packer.device)
  _lib.check(L.lddl_render_npy(*args, _ptr(data), nb.value, ctypes.byref(nb), s))
  if not host:
    return off, data[:nb.value]
  return _host(off, stream), _host(data[:nb.value], stream)


def _npy_header(k):
  b = io.BytesIO()
  np.save(b, np.zeros(k, dtype=np.uint16))  # serialize_np_array, lddl/utils.py:98-102
  return np.frombuffer(b.getvalue()[:len(b.getvalue()) - 2 * k], dtype=np.uint8)


def npy_positions(mlm_off, mlm_pos):
  """masked_lm_positions column: per row the np.save bytes of uint16[k]
  (header + 2k bytes), built vectorised.  mlm_off: int64[n+1] (from 0),
  mlm_pos: uint16[mlm_off[-1]].  Returns (int64 offsets, uint8 data)."""
  k = np.diff(mlm_off)
  uk, inv = np.unique(k, return_inverse=True)
  hdr = [_npy_header(int(v)) for v in uk]
  if len(k) and len({len(h) for h in hdr}) == 1 and len(hdr[0]) % 2 == 0:
    return _npy_positions_u16(k, inv, hdr, mlm_pos)
  hdr = dict(zip((int(v) for v in uk), hdr))
  hlen = np.array([len(hdr[int(v)]) for v in k], dtype=np.int64) if len(k) else np.zeros(0, np.int64)
  sizes = hlen + 2 * k
  off = np.zeros(len(k) + 1, dtype=np.int64)
  np.cumsum(sizes, out=off[1:])
  data = np.empty(int(off[-1]), dtype=np.uint8)
  for v, h in hdr.items():
    rows = np.nonzero(k == v)[0]
    data[(off[rows][:, None] + np.arange(len(h))[None, :]).ravel()] = np.tile(h, len(rows))
  # position bytes: row r's 2k bytes start at off[r] + hlen[r]
  if len(mlm_pos):
    rix = np.repeat(np.arange(len(k)), 2 * k)
    within = np.arange(int(2 * k.sum())) - np.repeat(2 * mlm_off[:-1], 2 * k)
    data[off[rix] + hlen[rix] + within] = np.ascontiguousarray(mlm_pos, dtype='<u2').view(np.uint8)
  return off, data


def _npy_positions_u16(k, inv, hdr, mlm_pos):
  """npy_positions when every row's header has one even length H (np.save
  pads its v1.0 header to 128 bytes for any 1-D uint16 shape): the column is
  a u16 stream whose header slots are H/2 values at each row start, filled
  by two boolean-mask assignments instead of index arrays per byte."""
  h2 = len(hdr[0]) // 2
  sizes = h2 + k  # u16 units
  off16 = np.zeros(len(k) + 1, dtype=np.int64)
  np.cumsum(sizes, out=off16[1:])
  data = np.empty(int(off16[-1]), dtype='<u2')
  is_hdr = np.zeros(int(off16[-1]) + 1, dtype=np.int8)
  is_hdr[off16[:-1]] += 1  # (starts distinct, ends distinct: each pass has no repeated index)
  is_hdr[off16[:-1] + h2] -= 1
  is_hdr = np.cumsum(is_hdr[:-1], dtype=np.int8).view(bool)
  table = np.stack([np.frombuffer(h.tobytes(), dtype='<u2') for h in hdr])
  data[is_hdr] = table[inv].ravel()
  data[~is_hdr] = np.ascontiguousarray(mlm_pos, dtype='<u2')
  return off16 * 2, data.view(np.uint8)


# Arrow arrays straight from buffers: pa.array() on numpy arrays or Python
# lists imports pandas on its first call (~0.4-0.5 s per process)
_NP_TYPES = {np.dtype(np.uint16): pa.uint16(), np.dtype(np.int64): pa.int64(), np.dtype(np.int32): pa.int32()}


def np_array(x):
  """Arrow array of a 1-D numpy array (bool, uint16, int32 or int64), no copy
  except bools (bit-packed)"""
  x = np.ascontiguousarray(x)
  if x.dtype == np.bool_:
    return pa.Array.from_buffers(pa.bool_(), len(x), [None, pa.py_buffer(np.packbits(x, bitorder='little'))])
  return pa.Array.from_buffers(_NP_TYPES[x.dtype], len(x), [None, pa.py_buffer(x)])


def str_array(strs):
  """Arrow string array of a list of str"""
  b = [s.encode('utf-8') for s in strs]
  off = np.zeros(len(b) + 1, dtype=np.int64)
  np.cumsum(np.fromiter(map(len, b), dtype=np.int64, count=len(b)), out=off[1:])
  return _arrow(pa.string(), off, np.frombuffer(b''.join(b), dtype=np.uint8), 0, len(b))


OFF32_LIMIT = 2**31


def _arrow_rows(typ, off, data, n):
  """all n rows of a (int64 offsets from 0, bytes) column: 32-bit offsets, or
  the large type when the bytes pass 2 GiB (files slice and cast it)"""
  if off[n] < OFF32_LIMIT:
    return pa.Array.from_buffers(typ, n, [None, pa.py_buffer(off[:n + 1].astype(np.int32)), pa.py_buffer(data)])
  big = pa.large_string() if typ == pa.string() else pa.large_binary()
  return pa.Array.from_buffers(big, n, [None, pa.py_buffer(np.ascontiguousarray(off[:n + 1])), pa.py_buffer(data)])


def _arrow(typ, off, data, lo, hi):
  """rows [lo, hi) of a (int64 offsets, bytes) column as an Arrow array"""
  o = off[lo:hi + 1] - off[lo]
  d = data[off[lo]:off[hi]]
  if o[-1] < 2**31:
    return pa.Array.from_buffers(typ, hi - lo, [None, pa.py_buffer(o.astype(np.int32)), pa.py_buffer(d)])
  big = pa.large_string() if typ == pa.string() else pa.large_binary()
  return pa.Array.from_buffers(big, hi - lo, [None, pa.py_buffer(o), pa.py_buffer(d)]).cast(typ)


def file_table(sch, cols, raw, lo, hi, batch=None):
  """rows [lo, hi) of a writer batch as one file's table.  batch: the batch's
  table when every column fits its schema type (a zero-copy slice of it);
  otherwise (a string column's batch bytes pass 2 GiB: large_string) each
  string column is rebuilt from raw[name] = (type, int64 offsets, bytes)
  with offsets rebased to the file's first row -- a slice of the large
  column keeps absolute offsets, which a cast back to string rejects past
  2^31 (the file's own bytes fit)"""
  if batch is not None:
    return batch.slice(lo, hi - lo)
  arrs = [_arrow(*raw[nm], lo, hi) if nm in raw else cols[nm].slice(lo, hi - lo) for nm in sch.names]
  return pa.Table.from_arrays(arrs, schema=sch)


def _worker_init():
  from . import encode_worker  # noqa: F401  (imported before the first batch)
  n = int(os.environ.get('LDDL_WORKER_NICE', '5'))  # (niced as the CLI's split workers)
  if n > 0:
    try:
      os.nice(n)
    except OSError:
      pass


def _warm(_):
  return os.getpid()


class ProcessEncoder:
  """Parquet encodes in a pool of host processes (encode_worker.encode).

  The per-file part of pyarrow's writer holds the GIL, so a thread pool
  serialises on small files (CodeBERT's, ~100 rows each); processes each
  have their own.  A batch's columns are copied once into a shared slot
  file under /dev/shm (device columns straight from the GPU, through the
  slot pinned with hipHostRegister when the runtime allows), then each task
  writes a run of the batch's files from it.  `slots` batches can be in
  flight; a slot is reused once its batch's files are written.  Create it
  before the process touches the GPU (its workers are forked); close() ends
  the workers and removes the slot files."""

  def __init__(self, workers=None, slots=3, context='fork'):
    import multiprocessing as mp
    self.workers = workers or encode_workers()
    self.ex = concurrent.futures.ProcessPoolExecutor(self.workers, mp_context=mp.get_context(context),
                                                     initializer=_worker_init)
    list(self.ex.map(_warm, range(self.workers)))  # start the workers now, not in the first batch
    d = None
    if os.path.isdir('/dev/shm') and os.access('/dev/shm', os.W_OK):
      st = os.statvfs('/dev/shm')
      if st.f_bavail * st.f_frsize >= (1 << 30) * slots:  # (a small /dev/shm would fault on the slot writes)
        d = '/dev/shm'
    import tempfile
    self.dir = tempfile.mkdtemp(prefix='lddl_enc_', dir=d)
    self.slots = [dict(path=os.path.join(self.dir, 'slot%d' % i), size=0, mm=None, t=None, pinned=False, futs=[])
                  for i in range(slots)]
    self.disk_dir = None  # (slots that outgrew /dev/shm: _grow)
    self.next = 0
    self.wait_s = 0.0  # waiting for a slot's previous batch to finish encoding
    self.copy_s = 0.0  # columns into the slots (device copies included)
    # the slot files are memory: removed at exit even when close() is never
    # reached (an exception on the caller's path)
    import shutil
    import weakref
    self._fin = weakref.finalize(self, shutil.rmtree, self.dir, True)

  def submit(self, fn, *a, **kw):  # (a plain task, as an executor)
    return self.ex.submit(fn, *a, **kw)

  def _unpin(self, sl):
    if sl['pinned']:
      torch.cuda.cudart().cudaHostUnregister(sl['t'].data_ptr())
      sl['pinned'] = False

  def _grow(self, sl, new):
    """The slot file at `new` bytes, its space reserved (posix_fallocate), so
    a full tmpfs is an OSError here and not a SIGBUS in the copy into the
    mapping (the /dev/shm check at construction sees neither the slots'
    growth nor the other ranks of the node).  A slot that no longer fits in
    /dev/shm moves to a directory on disk."""
    import errno
    import mmap
    for attempt in range(2):
      fd = os.open(sl['path'], os.O_RDWR | os.O_CREAT, 0o600)
      try:
        os.ftruncate(fd, new)
        try:
          os.posix_fallocate(fd, 0, new)
        except OSError as e:
          if e.errno not in (errno.ENOSPC, errno.EFBIG, errno.EDQUOT) or attempt:
            raise OSError(e.errno, 'parquet encoder slot of %d MB: no space in %s (%s)' % (
                new >> 20, os.path.dirname(sl['path']), e.strerror)) from e
          os.ftruncate(fd, 0)
          if self.disk_dir is None:
            import shutil
            import tempfile
            import weakref
            self.disk_dir = tempfile.mkdtemp(prefix='lddl_enc_')
            self._fin_disk = weakref.finalize(self, shutil.rmtree, self.disk_dir, True)
          os.close(fd)
          fd = -1
          os.remove(sl['path'])
          sl['path'] = os.path.join(self.disk_dir, os.path.basename(sl['path']))
          continue
        return mmap.mmap(fd, new)
      finally:
        if fd >= 0:
          os.close(fd)

  def _acquire(self, size):
    sl = self.slots[self.next]
    self.next = (self.next + 1) % len(self.slots)
    t0 = time.perf_counter()
    for f_ in sl['futs']:
      f_.result()
    self.wait_s += time.perf_counter() - t0
    sl['futs'] = []
    if sl['size'] < size:
      import mmap
      self._unpin(sl)
      sl['t'] = None
      if sl['mm'] is not None:
        sl['mm'].close()
      new = max(size, 2 * sl['size'], 64 << 20)
      new = (new + (1 << 21) - 1) & ~((1 << 21) - 1)
      sl['mm'] = self._grow(sl, new)
      sl['size'] = new
      sl['t'] = torch.frombuffer(sl['mm'], dtype=torch.uint8)
      if torch.cuda.is_initialized():
        try:
          sl['pinned'] = torch.cuda.cudart().cudaHostRegister(sl['t'].data_ptr(), new, 0) == 0
        except Exception:  # (not available: pageable copies)
          sl['pinned'] = False
    return sl

  def submit_batch(self, n, specs, sch, files, compression, dict_cols, stream=None):
    """specs: (name, kind, a, b) per schema column: 'str' / 'bin' with
    a = int64 offsets [n + 1] from 0 and b = bytes (device tensors or numpy),
    or 'bool' / 'u16' / 'i64' with a = numpy values [n]; files: (path, lo, hi)
    row ranges.  Returns the tasks' futures."""
    def nbytes(x):
      return x.numel() * x.element_size() if isinstance(x, torch.Tensor) else x.nbytes

    lay, pos = [], 0
    for name, kind, a, b in specs:
      p0 = (pos + 63) & ~63
      if kind in ('str', 'bin'):
        p1 = (p0 + nbytes(a) + 63) & ~63
        lay.append((name, kind, p0, p1))
        pos = p1 + nbytes(b)
      else:
        lay.append((name, kind, p0, 0))
        pos = p0 + nbytes(a)
    sl = self._acquire(max(pos, 64))
    t0 = time.perf_counter()
    dst = sl['t']
    dev = False
    st = None
    for (name, kind, a, b), (_, _, p0, p1) in zip(specs, lay):
      for x, at in ((a, p0), (b, p1)) if kind in ('str', 'bin') else ((a, p0),):
        k = nbytes(x)
        if k == 0:
          continue
        if isinstance(x, torch.Tensor):
          st = st or stream or torch.cuda.current_stream()
          with torch.cuda.stream(st):  # (the copies on the stream the columns were rendered on)
            dst[at:at + k].copy_(x.reshape(-1).view(torch.uint8), non_blocking=sl['pinned'])
          dev = True
        else:
          dst[at:at + k].numpy()[:] = np.ascontiguousarray(x).reshape(-1).view(np.uint8)
    if dev:
      st.synchronize()
    self.copy_s += time.perf_counter() - t0
    from . import encode_worker
    # tasks of about equal rows, at least one file each, ~2 per worker
    ntask = max(1, min(len(files), 2 * self.workers))
    bounds = np.searchsorted(np.array([f_[2] for f_ in files]), np.linspace(0, n, ntask + 1)[1:-1], side='left')
    cuts = [0] + sorted(set(int(x) + 1 for x in bounds if 0 <= x < len(files) - 1)) + [len(files)]
    cols = [(name, kind, p0, p1) for name, kind, p0, p1 in lay]
    futs = [self.ex.submit(encode_worker.encode, sl['path'], sl['size'], n, cols, sch, files[a:b], compression,
                           dict_cols) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
    sl['futs'] = list(futs)
    return futs

  def close(self):
    for sl in self.slots:
      for f_ in sl['futs']:
        try:
          f_.result()
        except Exception:
          pass
    t0 = time.perf_counter()
    self.ex.shutdown(wait=True)
    t1 = time.perf_counter()
    for sl in self.slots:
      self._unpin(sl)
      sl['t'] = None
      if sl['mm'] is not None:
        sl['mm'].close()
        sl['mm'] = None
    t2 = time.perf_counter()
    self._fin()
    if self.disk_dir is not None:
      self._fin_disk()
    self.close_s = (t1 - t0, t2 - t1, time.perf_counter() - t2)  # workers' exit, slot unpin / unmap, slot files


def _host_var(arr, r0, n):
  """rows [r0, r0 + n) of an Arrow string array as (int64 offsets from 0, bytes)"""
  a = arr.slice(r0, n)
  wide = a.type in (pa.large_string(), pa.large_binary())
  off = np.frombuffer(a.buffers()[1], dtype=np.int64 if wide else np.int32, count=a.offset + n + 1)[a.offset:]
  off = off.astype(np.int64)
  buf = a.buffers()[2]
  # (Arrow may leave the data buffer out when every string of the slice is empty)
  data = np.frombuffer(buf, dtype=np.uint8, count=int(off[-1]))[int(off[0]):] if n and buf is not None and off[-1] \
      else np.zeros(0, np.uint8)
  return off - off[0], data


LAST_STATS = {}  # the last write_shards call's stage seconds (bench.py reports them)


def write_shards(packer, res, out_dir, bin_size=None, codebert=False, masking=False, doc_ids=None,
                 part_base=0, compression='snappy', batch_rows=1 << 16, max_parts=None, stream=None,
                 executor=None, pending=None):
  """Write the rows of ``res`` (a pipeline.PackResult) as the reference's
  parquet files under out_dir.  Partition p of this pack call is file
  ``part.{part_base + p}.parquet`` (unbinned) or ``part.{..}.parquet_{b}``
  for every bin b (binned).  doc_ids: CodeBERT 'id' strings (list or Arrow array) per document of
  the packed corpus.  max_parts: only the first max_parts partitions.
  executor / pending: the parquet encodes go to the caller's thread pool and
  their futures to the caller's list, and this call returns once the string
  columns are rendered and on the host (the device buffers are free again):
  the encodes run on while the caller's next chunk splits and packs.
  Rows are rendered in batches of whole files of about batch_rows rows, so
  the files of one batch encode while the next renders.
  Returns the list of files (written once the futures are done)."""
  t_start = time.perf_counter()
  os.makedirs(out_dir, exist_ok=True)
  binned = bin_size is not None
  nbins = res.nbins if binned else 1
  n_part = res.bin_count.shape[0]
  counts = res.bin_count.cpu().numpy().reshape(n_part, res.nbins)
  if not binned:
    counts = counts.sum(axis=1, keepdims=True)
  file_rows = counts.ravel()  # (partition, bin) major order == row order
  file_start = np.zeros(len(file_rows) + 1, dtype=np.int64)
  np.cumsum(file_rows, out=file_start[1:])
  assert file_start[-1] == res.n_pairs, (file_start[-1], res.n_pairs)
  sch = schema(codebert, masking and not codebert, binned)
  # dictionary pages only where values repeat (flags, lengths, bins, the
  # CodeBERT id of a document's rows): the segment / label strings are unique
  # per row and the encoder would build and then discard a dictionary for them
  dict_cols = [n_ for n_ in sch.names if n_ not in DENSE_COLS]
  nfiles = len(file_rows) if max_parts is None else min(len(file_rows), max_parts * nbins)
  n_rows = int(file_start[nfiles])  # rows of the files written
  num_tokens = np.diff(res.tok_off[:n_rows + 1].cpu().numpy()).astype(np.uint16)
  flags = res.flags[:n_rows].cpu().numpy()
  bins = res.bins[:n_rows].cpu().numpy().astype(np.int64)
  docs = None
  if codebert:
    if doc_ids is None:
      raise ValueError('CodeBERT shards need doc_ids (the id column)')
    docs = np_array(row_docs(packer, res, n_rows, stream))
    ids_arr = doc_ids if isinstance(doc_ids, pa.Array) else str_array(doc_ids)
    ids_col = ids_arr.take(docs) if n_rows else str_array([])
  host_mlm = []  # (offsets, positions) on the host, fetched only for the host npy path

  def mlm_host():
    if not host_mlm:
      moff = res.mlm_off[:n_rows + 1].cpu().numpy()
      host_mlm.extend([moff, res.mlm_pos[:int(moff[-1])].cpu().numpy().view(np.uint16)])
    return host_mlm
  files = []
  f = 0
  workers = encode_workers()
  st = {'setup_s': time.perf_counter() - t_start, 'render_s': 0.0, 'table_s': 0.0, 'backpressure_s': 0.0,
        'drain_s': 0.0, 'batches': 0, 'workers': workers}
  own = executor is None
  proc = isinstance(executor, ProcessEncoder)
  if proc:
    st['workers'] = executor.workers
  pool = concurrent.futures.ThreadPoolExecutor(workers) if own else executor
  mine = []
  # render in batches of whole files (>= batch_rows rows, or one big file)
  while f < nfiles:
    g = f + 1
    while g < nfiles and file_start[g + 1] - file_start[f] <= batch_rows:
      g += 1
    r0, r1 = int(file_start[f]), int(file_start[g])
    n = r1 - r0
    t0 = time.perf_counter()
    if proc:
      c0, c1 = seg_columns(packer, res, r0, n, codebert, stream, host=False)
      var = {('doc' if codebert else 'A'): c0, ('code' if codebert else 'B'): c1}
      if masking and not codebert:
        var['masked_lm_labels'] = render(packer, res.mlm_label, res.mlm_off, r0, n, ROW, stream=stream, host=False)
        pos = render_npy(packer, res, r0, n, stream, host=False)
        if pos is None:
          moff_all, mpos_all = mlm_host()
          m0 = int(moff_all[r0])
          pos = npy_positions(moff_all[r0:r1 + 1] - m0, mpos_all[m0:int(moff_all[r1])])
        var['masked_lm_positions'] = pos
      if codebert:
        var['id'] = _host_var(ids_col, r0, n)
      fixed = {'is_random_next': ('bool', (flags[r0:r1] & 1).astype(bool)), 'num_tokens': ('u16', num_tokens[r0:r1]),
               'bin_id': ('i64', bins[r0:r1])}
      specs = [(nm, 'bin' if nm == 'masked_lm_positions' else 'str') + tuple(var[nm]) if nm in var else
               (nm, fixed[nm][0], fixed[nm][1], None) for nm in sch.names]
      flist = []
      for fi in range(f, g):
        p, b = divmod(fi, nbins)
        name = 'part.%d.parquet' % (part_base + p)
        if binned:
          name += '_%d' % b
        flist.append((os.path.join(out_dir, name), int(file_start[fi] - r0), int(file_start[fi + 1] - r0)))
      t1 = time.perf_counter()
      st['render_s'] += t1 - t0
      st['batches'] += 1
      mine.extend(executor.submit_batch(n, specs, sch, flist, compression, dict_cols, stream))
      files.extend(f_[0] for f_ in flist)
      st['table_s'] += time.perf_counter() - t1
      f = g
      continue
    c0, c1 = seg_columns(packer, res, r0, n, codebert, stream)
    if masking and not codebert:
      lab = render(packer, res.mlm_label, res.mlm_off, r0, n, ROW, stream=stream)
      pos = render_npy(packer, res, r0, n, stream)
      if pos is None:
        moff_all, mpos_all = mlm_host()
        m0 = int(moff_all[r0])
        pos = npy_positions(moff_all[r0:r1 + 1] - m0, mpos_all[m0:int(moff_all[r1])])
    t1 = time.perf_counter()
    st['render_s'] += t1 - t0
    st['batches'] += 1
    # one table over the batch's rows; a file is a zero-copy slice of it
    cols, raw = {}, {}
    if codebert:
      cols['id'] = ids_col.slice(r0, n)
      raw['doc'], raw['code'] = (pa.string(),) + tuple(c0), (pa.string(),) + tuple(c1)
    else:
      raw['A'], raw['B'] = (pa.string(),) + tuple(c0), (pa.string(),) + tuple(c1)
      cols['is_random_next'] = np_array((flags[r0:r1] & 1).astype(bool))
    cols['num_tokens'] = np_array(num_tokens[r0:r1])
    if masking and not codebert:
      raw['masked_lm_positions'] = (pa.binary(),) + tuple(pos)
      raw['masked_lm_labels'] = (pa.string(),) + tuple(lab)
    if binned:
      cols['bin_id'] = np_array(bins[r0:r1])
    for nm, (typ, off, data) in raw.items():
      cols[nm] = _arrow_rows(typ, off, data, n)
    arrs = [cols[name] for name in sch.names]
    large = any(a.type != fd.type for a, fd in zip(arrs, sch))
    tb = None if large else pa.Table.from_arrays(arrs, names=sch.names)
    for fi in range(f, g):
      lo, hi = int(file_start[fi] - r0), int(file_start[fi + 1] - r0)
      p, b = divmod(fi, nbins)
      t = file_table(sch, cols, raw, lo, hi, tb)
      name = 'part.%d.parquet' % (part_base + p)
      if binned:
        name += '_%d' % b
      path = os.path.join(out_dir, name)
      mine.append(pool.submit(pq.write_table, t, path, compression=compression, use_dictionary=dict_cols))
      files.append(path)
    t2 = time.perf_counter()
    st['table_s'] += t2 - t1
    # the parquet encoder releases the GIL: files of a batch encode in
    # parallel on the host cores while the next batch renders on the GPU
    while len(mine) > 4 * workers:
      mine.pop(0).result()
    st['backpressure_s'] += time.perf_counter() - t2
    f = g
  t3 = time.perf_counter()
  if own:
    for fu in mine:
      fu.result()
    pool.shutdown()
  else:
    pending.extend(mine)
  st['drain_s'] = time.perf_counter() - t3
  st['total_s'] = time.perf_counter() - t_start
  LAST_STATS.clear()
  LAST_STATS.update(st)
  return files


def encode_workers():
  """parquet encode threads: the host CPU share (hostinfo.cpu_share), or
  LDDL_ENCODE_WORKERS"""
  e = os.environ.get('LDDL_ENCODE_WORKERS')
  if e:
    return max(1, int(e))
  from .hostinfo import cpu_share
  return cpu_share()


def write_txt(packer, res, out_dir, bin_size=None, codebert=False, masking=False, doc_ids=None, part_base=0,
              batch_rows=1 << 20, max_parts=None, stream=None):
  """The reference's txt sink (--output-format txt, pretrain.py:501-531,
  pretrain_codebert.py:540-559): one line per row,

    BERT      is_random_next: {b} - [CLS] {A} [SEP] {B} [SEP] - {num_tokens}
    masking   is_random_next: {b} - [CLS] {A} [SEP] {B} [SEP] - masked_lm_positions: {str(np.array)}
              - masked_lm_labels: {labels} - {num_tokens}
    CodeBERT  {id} [CLS] {doc} [SEP] {code} [SEP] - {num_tokens}

  joined by '\\n' with no final newline (dask's to_textfiles).  Files:
  {p}.txt per partition (to_textfiles' default name), or {p}_{b}.txt for
  every bin b (binning.py:439-476: the bin parsed back from the line's last
  field, rows in shuffled order within a bin == this packer's row order).
  Every file is created, empty ones included.  Returns the files."""
  os.makedirs(out_dir, exist_ok=True)
  binned = bin_size is not None
  nbins = res.nbins if binned else 1
  n_part = res.bin_count.shape[0]
  counts = res.bin_count.cpu().numpy().reshape(n_part, res.nbins)
  if not binned:
    counts = counts.sum(axis=1, keepdims=True)
  file_rows = counts.ravel()
  file_start = np.zeros(len(file_rows) + 1, dtype=np.int64)
  np.cumsum(file_rows, out=file_start[1:])
  nfiles = len(file_rows) if max_parts is None else min(len(file_rows), max_parts * nbins)
  n_rows = int(file_start[nfiles])
  num_tokens = np.diff(res.tok_off[:n_rows + 1].cpu().numpy())
  flags = res.flags[:n_rows].cpu().numpy()
  if codebert:
    if doc_ids is None:
      raise ValueError('CodeBERT txt output needs doc_ids (the id field)')
    if isinstance(doc_ids, pa.Array):
      doc_ids = doc_ids.to_pylist()
    docs = row_docs(packer, res, n_rows, stream)
  if masking and not codebert:
    moff_all = res.mlm_off[:n_rows + 1].cpu().numpy()
    mpos_all = res.mlm_pos[:int(moff_all[-1])].cpu().numpy().view(np.uint16)
  files = []
  f = 0
  while f < nfiles:
    g = f + 1
    while g < nfiles and file_start[g + 1] - file_start[f] <= batch_rows:
      g += 1
    r0, r1 = int(file_start[f]), int(file_start[g])
    n = r1 - r0
    (o0, d0), (o1, d1) = seg_columns(packer, res, r0, n, codebert, stream)
    if masking and not codebert:
      ol, dl = render(packer, res.mlm_label, res.mlm_off, r0, n, ROW, stream=stream)
    b0, b1 = d0.tobytes(), d1.tobytes()
    bl = dl.tobytes() if masking and not codebert else b''
    for fi in range(f, g):
      lo, hi = int(file_start[fi] - r0), int(file_start[fi + 1] - r0)
      p, b = divmod(fi, nbins)
      lines = []
      for i in range(lo, hi):
        r = r0 + i
        a, bb = b0[o0[i]:o0[i + 1]].decode(), b1[o1[i]:o1[i + 1]].decode()
        if codebert:
          lines.append('{} [CLS] {} [SEP] {} [SEP] - {}'.format(doc_ids[docs[r]], a, bb, int(num_tokens[r])))
        elif masking:
          pos = np.array(mpos_all[moff_all[r] - moff_all[0]:moff_all[r + 1] - moff_all[0]], dtype=np.uint16)
          lines.append('is_random_next: {} - [CLS] {} [SEP] {} [SEP] - masked_lm_positions: {} - '
                       'masked_lm_labels: {} - {}'.format(bool(flags[r] & 1), a, bb, pos,
                                                          bl[ol[i]:ol[i + 1]].decode(), int(num_tokens[r])))
        else:
          lines.append('is_random_next: {} - [CLS] {} [SEP] {} [SEP] - {}'.format(bool(flags[r] & 1), a, bb,
                                                                                 int(num_tokens[r])))
      name = ('%d_%d.txt' % (part_base + p, b)) if binned else ('%d.txt' % (part_base + p))
      path = os.path.join(out_dir, name)
      with open(path, 'w', encoding='utf-8', newline='') as fh:
        fh.write('\n'.join(lines))
      files.append(path)
    f = g
  return files
