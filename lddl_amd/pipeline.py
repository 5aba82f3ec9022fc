"""Host side of the hot path: tokenize -> pack -> bin -> materialise on one GPU.

Mirrors the reference's per-partition callbacks
(``_get_documents._to_document`` pretrain.py:82-97 and
``_get_pairs._to_partition_pairs`` :386-402, ``_to_dataframe_binned``
binning.py:63-93) over a whole set of partitions at once.  All compute runs in
liblddl_amd.so; this module only moves buffers and calls the C-ABI.

A *shard set* is a sentence-split corpus resident in HBM:
  data          uint8  [nbytes + 16]   UTF-8 sentences back to back
  sent_off      int64  [n_sent + 1]
  doc_sent_off  int64  [n_doc + 1]
  part_doc_off  int64  [n_part + 1]    partition = consecutive documents
  doc_nseg_doc  int32  [n_doc]         CodeBERT only: leading docstring segments
Partition p is packed after random.seed(seed + p) (the reference leaves the
partition RNG unseeded).
"""
import ctypes
import dataclasses

import numpy as np
import torch

from . import _lib
from .tokenizer import Tokenizer, _ptr, _stream

VOCAB_BERT = _lib.VOCAB_BERT
VOCAB_CODEBERT = _lib.VOCAB_CODEBERT


def partition_by_bytes(corpus, n_partitions):
  """part_doc_off splitting documents into n_partitions of ~equal bytes
  (the reference sizes Dask partitions by bytes: --block-size/--num-blocks,
  readers.py:48-57)."""
  n_doc = corpus.n_doc
  n_partitions = max(1, min(n_partitions, max(1, n_doc)))
  doc_bytes = corpus.sent_off[corpus.doc_sent_off[1:]] - corpus.sent_off[corpus.doc_sent_off[:-1]]
  cum = np.concatenate([[0], np.cumsum(doc_bytes)])
  cuts = np.searchsorted(cum, np.linspace(0, cum[-1], n_partitions + 1)[1:-1])
  off = np.concatenate([[0], cuts, [n_doc]]).astype(np.int64)
  off = np.maximum.accumulate(off)
  return off


@dataclasses.dataclass
class ShardSet:
  data: torch.Tensor
  sent_off: torch.Tensor
  doc_sent_off: torch.Tensor
  part_doc_off: torch.Tensor
  doc_nseg_doc: torch.Tensor = None
  nbytes: int = 0

  @property
  def n_sent(self):
    return self.sent_off.numel() - 1

  @property
  def n_doc(self):
    return self.doc_sent_off.numel() - 1

  @property
  def n_part(self):
    return self.part_doc_off.numel() - 1


def upload(corpus, part_doc_off, device):
  part_doc_off = np.asarray(part_doc_off, dtype=np.int64)
  if part_doc_off[0] != 0 or part_doc_off[-1] != corpus.n_doc or np.any(np.diff(part_doc_off) < 0):
    raise ValueError('part_doc_off must be a non-decreasing cover of [0, n_doc]')
  if np.any(np.diff(corpus.doc_sent_off) < 0) or np.any(np.diff(corpus.sent_off) < 0):
    raise ValueError('offsets must be non-decreasing')
  # pinned staging + async H2D on the current stream (ordered before the
  # tokenize launch; the caching host allocator keeps the staging buffers
  # until the copies have run)
  def h2d(a):
    return torch.from_numpy(np.ascontiguousarray(a)).pin_memory().to(device, non_blocking=True)

  data = torch.empty(corpus.nbytes + 16, dtype=torch.uint8, device=device)
  data[:corpus.nbytes].copy_(torch.from_numpy(np.ascontiguousarray(corpus.data[:corpus.nbytes])).pin_memory(),
                             non_blocking=True)
  data[corpus.nbytes:].zero_()
  nseg = None
  if corpus.doc_nseg_doc is not None:
    nseg = h2d(np.asarray(corpus.doc_nseg_doc, dtype=np.int32))
  return ShardSet(data, h2d(corpus.sent_off - corpus.sent_off[0]), h2d(corpus.doc_sent_off), h2d(part_doc_off), nseg,
                  corpus.nbytes)


def upload_pieces(corpora, part_doc_off, device):
  """upload() of consecutive corpus pieces (a chunk split on several host
  workers) without concatenating them on the host first: each piece is
  copied once, straight into the pinned staging buffers of the H2D copies."""
  if len(corpora) == 1:
    return upload(corpora[0], part_doc_off, device)
  part_doc_off = np.asarray(part_doc_off, dtype=np.int64)
  NB = sum(c.nbytes for c in corpora)
  NS = sum(c.n_sent for c in corpora)
  ND = sum(c.n_doc for c in corpora)
  if part_doc_off[0] != 0 or part_doc_off[-1] != ND or np.any(np.diff(part_doc_off) < 0):
    raise ValueError('part_doc_off must be a non-decreasing cover of [0, n_doc]')
  data_h = torch.empty(max(NB, 1), dtype=torch.uint8, pin_memory=True)
  so_h = torch.empty(NS + 1, dtype=torch.int64, pin_memory=True)
  dso_h = torch.empty(ND + 1, dtype=torch.int64, pin_memory=True)
  dv, sv, dsv = data_h.numpy(), so_h.numpy(), dso_h.numpy()
  sv[0] = dsv[0] = 0
  b = ns = nd = 0
  for c in corpora:
    if np.any(np.diff(c.doc_sent_off) < 0) or np.any(np.diff(c.sent_off) < 0):
      raise ValueError('offsets must be non-decreasing')
    s0 = int(c.sent_off[0])
    dv[b:b + c.nbytes] = c.data[s0:s0 + c.nbytes]
    np.add(c.sent_off[1:], b - s0, out=sv[ns + 1:ns + 1 + c.n_sent])
    np.add(c.doc_sent_off[1:], ns - int(c.doc_sent_off[0]), out=dsv[nd + 1:nd + 1 + c.n_doc])
    b += c.nbytes
    ns += c.n_sent
    nd += c.n_doc
  data = torch.empty(NB + 16, dtype=torch.uint8, device=device)
  data[:NB].copy_(data_h[:NB], non_blocking=True)
  data[NB:].zero_()
  nseg = None
  if corpora[0].doc_nseg_doc is not None:
    nseg = torch.from_numpy(np.concatenate([c.doc_nseg_doc for c in corpora]).astype(np.int32)).pin_memory().to(
        device, non_blocking=True)
  h2d = lambda t: t.to(device, non_blocking=True)  # noqa: E731
  return ShardSet(data, h2d(so_h), h2d(dso_h), h2d(torch.from_numpy(part_doc_off).pin_memory()), nseg, NB)


@dataclasses.dataclass
class PackResult:
  n_pairs: int
  n_tokens: int
  nbins: int
  tokens: torch.Tensor     # int16 view of uint16 ids, rows back to back
  tok_off: torch.Tensor    # int64 [n_pairs + 1]
  len0: torch.Tensor       # int16 view of uint16
  len1: torch.Tensor
  flags: torch.Tensor      # uint8
  bins: torch.Tensor       # uint8
  part: torch.Tensor       # int64
  bin_count: torch.Tensor  # int64 [n_part, nbins]
  ids: torch.Tensor = None       # the tokenizer's dense ids (sentence s at ids_off[s])
  ntok: torch.Tensor = None
  ids_off: torch.Tensor = None
  n_masked: int = 0
  mlm_off: torch.Tensor = None    # int64 [n_pairs + 1] (masking only)
  mlm_pos: torch.Tensor = None    # int16 view of uint16 positions (row coordinates)
  mlm_label: torch.Tensor = None  # int16 view of uint16 label ids
  ntok_host: np.ndarray = None
  part_doc_off: np.ndarray = None
  mlm_token: torch.Tensor = None  # spans + masking: int16 view of the token each masked position shows
  src0: torch.Tensor = None       # spans (lddl_row_spans): int64 [n_pairs] dense-id offset of A / doc
  src1: torch.Tensor = None       # of B / code; tokens is then None (no rows materialised)
  cls_id: int = 0
  sep_id: int = 0
  pack: 'PackHandle' = None       # the lddl_pack this result was packed into (lddl_row_docs reads it)

  @property
  def spans(self):
    return self.src0 is not None

  def host_tokens(self):
    """the rows back to back on the host (int64), from the materialised
    rows or rebuilt from the spans over the dense ids"""
    if not self.spans:
      return self.tokens[:self.n_tokens].cpu().numpy().view(np.uint16).astype(np.int64)
    n = self.n_pairs
    ids = self.ids.cpu().numpy().view(np.uint16).astype(np.int64)
    s0, s1 = self.src0[:n].cpu().numpy(), self.src1[:n].cpu().numpy()
    l0 = self.len0[:n].cpu().numpy().view(np.uint16).astype(np.int64)
    l1 = self.len1[:n].cpu().numpy().view(np.uint16).astype(np.int64)
    fl = self.flags[:n].cpu().numpy()
    if self.mlm_token is not None:  # the masked rows show mlm_token at mlm_pos
      moff = self.mlm_off[:n + 1].cpu().numpy()
      mpos = self.mlm_pos[:self.n_masked].cpu().numpy().view(np.uint16).astype(np.int64)
      mtok = self.mlm_token[:self.n_masked].cpu().numpy().view(np.uint16).astype(np.int64)
    out = []
    for g in range(n):
      a = ids[s0[g]:s0[g] + l0[g]]
      b = ids[s1[g]:s1[g] + l1[g]]
      sep0 = [self.sep_id] if fl[g] & 2 else []
      row = np.concatenate([[self.cls_id], a, sep0, b, [self.sep_id]]).astype(np.int64)
      if self.mlm_token is not None:
        row[mpos[moff[g]:moff[g + 1]]] = mtok[moff[g]:moff[g + 1]]
      out.append(row)
    return np.concatenate(out) if out else np.zeros(0, np.int64)

  def rows(self):
    """host copy: list of (partition, A ids, B ids, flags, bin)"""
    tok = self.host_tokens()
    off = self.tok_off[:self.n_pairs + 1].cpu().numpy()
    l0 = self.len0[:self.n_pairs].cpu().numpy().view(np.uint16).astype(np.int64)
    l1 = self.len1[:self.n_pairs].cpu().numpy().view(np.uint16).astype(np.int64)
    fl = self.flags[:self.n_pairs].cpu().numpy()
    bn = self.bins[:self.n_pairs].cpu().numpy()
    pt = self.part[:self.n_pairs].cpu().numpy()
    if self.mlm_off is not None:
      moff = self.mlm_off[:self.n_pairs + 1].cpu().numpy()
      mpos = self.mlm_pos[:self.n_masked].cpu().numpy().view(np.uint16).astype(np.int64)
      mlab = self.mlm_label[:self.n_masked].cpu().numpy().view(np.uint16).astype(np.int64)
    out = []
    for g in range(self.n_pairs):
      r = tok[off[g]:off[g + 1]]
      sep0 = bool(fl[g] & 2)
      a = r[1:1 + l0[g]]
      b = r[1 + l0[g] + (1 if sep0 else 0):1 + l0[g] + (1 if sep0 else 0) + l1[g]]
      row = (int(pt[g]), a.tolist(), b.tolist(), int(fl[g]), int(bn[g]), r.tolist())
      if self.mlm_off is not None:
        row += (mpos[moff[g]:moff[g + 1]].tolist(), mlab[moff[g]:moff[g + 1]].tolist())
      out.append(row)
    return out


class PackHandle:
  """A pack result (lddl_pack_new / lddl_pack_free): what one
  lddl_pack_bert / lddl_pack_codebert call leaves for the post-pack calls
  (lddl_materialize, lddl_row_spans, lddl_masked_lm[_spans],
  lddl_row_docs), which name it explicitly."""

  def __init__(self, tok):
    h = ctypes.c_void_p()
    _lib.check(_lib.lib().lddl_pack_new(tok.handle, ctypes.byref(h)))
    self._h = h.value
    self._out = {}  # the PackResult columns of packs into this handle (Packer._buf)

  @property
  def handle(self):
    return self._h

  def rows(self):
    """#rows of the last successful pack into it (-1: none)"""
    n = ctypes.c_int64()
    _lib.check(_lib.lib().lddl_pack_rows(self._h, ctypes.byref(n)))
    return n.value

  def close(self):
    if self._h:
      _lib.lib().lddl_pack_free(self._h)
      self._h = None

  def __del__(self):
    try:
      self.close()
    except Exception:
      pass


class TokBuffers:
  """A set of Packer.tokenize output buffers (ids, ntok, tok_off).  Passing
  alternating sets (bufs=) lets one batch's pack read its tokenizer output
  while the next batch tokenizes into the other set on another stream."""

  def __init__(self):
    self._out = {}


class Packer:
  """One GPU's tokenize -> pack -> bin -> materialise pipeline (one lddl_ctx
  and the pack result it packs into)."""

  def __init__(self, vocab_file=VOCAB_BERT, device=None, masking=False):
    self.tok = Tokenizer(vocab_file, device)
    if masking:  # the tokenizer records the [CLS]/[SEP] sentences the masked packer needs
      self.tok.set_special_flags(True)
    self.device = self.tok.device
    self.result = PackHandle(self.tok)
    self._out = {}

  def _buf(self, name, n, dtype, owner=None):
    """a cached device buffer of >= n entries; owner: the PackHandle whose
    PackResult columns it holds (each handle its own, so that several pack
    results stay live at once) or the TokBuffers of a tokenize call, else
    the Packer's own"""
    out = self._out if owner is None else owner._out
    t = out.get(name)
    if t is None or t.numel() < n or t.dtype != dtype:
      t = torch.empty(max(n, 1), dtype=dtype, device=self.device)
      out[name] = t
    return t

  @staticmethod
  def ids_estimate(nbytes):
    """ids buffer entries for a corpus of nbytes: WordPiece averages
    0.23 (Wikipedia-style) to 0.26 (code) tokens per byte; a denser input
    re-runs with the exact total (tokenize).  #tokens <= #bytes always."""
    return min(nbytes, nbytes * 3 // 8 + (1 << 16))

  def tokenize(self, shards, max_tok=512, stream=None, bufs=None):
    """-> (ids, ntok, tok_off): the dense CSR ids (lddl_tokenize).  The ids
    buffer is sized by ids_estimate, not by the byte count (20 GB of corpus:
    ~8 GB instead of 43 GB); the total is read back (one stream sync) and a
    corpus with more tokens runs again into a buffer of exactly its size.
    bufs: a TokBuffers to write into (default: the Packer's own buffers)."""
    from .tokenizer import CapacityError
    ntok = self._buf('ntok', shards.n_sent, torch.int32, bufs)
    toff = self._buf('tok_off_in', shards.n_sent + 1, torch.int64, bufs)
    cap = self.ids_estimate(shards.nbytes)
    for _ in range(2):
      ids = self._buf('ids', cap + 16, torch.int16, bufs)
      try:
        return self.tok.tokenize_device(shards.data, shards.sent_off, max_tok, ids, ntok, toff, stream,
                                        nbytes=shards.nbytes)
      except CapacityError as e:
        cap = e.total
    raise RuntimeError('lddl_amd: tokenize did not fit its exact total')

  def pack(self, shards, ids, ntok, tok_off=None, target_seq_length=128, short_seq_prob=0.1, duplicate_factor=5,
           seed=12345, bin_size=None, codebert=False, masking=False, masked_lm_ratio=0.15, stream=None,
           spans=False, into=None):
    """into: the PackHandle to pack into (default: the Packer's own).
    ids / ntok / tok_off: tokenize()'s dense CSR result (tok_off None:
    the exclusive scan of ntok, for ids built by hand); ids must hold 16
    entries of padding past the last id (lddl_materialize's 16-B loads).
    spans: the rows as spans of the dense ids (lddl_row_spans, no token
    copy; res.src0 / res.src1) instead of materialised rows -- what the
    parquet writer renders from; with masking, lddl_masked_lm_spans adds the
    token each masked position shows (res.mlm_token) in place of rewriting
    rows."""
    L = _lib.lib()
    if tok_off is None:
      tok_off = torch.zeros(shards.n_sent + 1, dtype=torch.int64, device=self.device)
      torch.cumsum(ntok[:shards.n_sent].to(torch.int64), 0, out=tok_off[1:])
    tot = (ctypes.c_int64 * 4)()
    s = _stream(stream)
    into = into or self.result
    h = into.handle
    if codebert:
      if shards.doc_nseg_doc is None:
        raise ValueError('CodeBERT packing needs doc_nseg_doc')
      rc = L.lddl_pack_codebert(self.tok.handle, h, _ptr(ntok), _ptr(tok_off), _ptr(shards.sent_off), shards.n_sent,
                                _ptr(shards.doc_sent_off), _ptr(shards.doc_nseg_doc), shards.n_doc,
                                _ptr(shards.part_doc_off), shards.n_part, target_seq_length, short_seq_prob,
                                duplicate_factor, abs(int(seed)), bin_size or 0, tot, s)
    else:
      rc = L.lddl_pack_bert(self.tok.handle, h, _ptr(ids) if masking else None, _ptr(ntok), _ptr(tok_off),
                            _ptr(shards.sent_off), shards.n_sent,
                            _ptr(shards.doc_sent_off), shards.n_doc, _ptr(shards.part_doc_off), shards.n_part,
                            target_seq_length, short_seq_prob, duplicate_factor, 1 if masking else 0,
                            masked_lm_ratio, abs(int(seed)), bin_size or 0, tot, s)
    if rc == -7:
      raise IndexError(L.lddl_last_error().decode())
    if rc == -8:
      raise AssertionError(L.lddl_last_error().decode())
    _lib.check(rc)
    n_pairs, n_tokens, nbins = int(tot[0]), int(tot[1]), int(tot[2])

    def buf(name, n, dtype):
      return self._buf(name, n, dtype, into)
    res = PackResult(n_pairs, n_tokens, nbins,
                     None if spans else buf('tokens', n_tokens, torch.int16),
                     buf('tok_off', n_pairs + 1, torch.int64),
                     buf('len0', n_pairs, torch.int16), buf('len1', n_pairs, torch.int16),
                     buf('flags', n_pairs, torch.uint8), buf('bins', n_pairs, torch.uint8),
                     buf('part', n_pairs, torch.int64),
                     buf('bin_count', shards.n_part * nbins, torch.int64))
    res.cls_id, res.sep_id = self.tok.cls_id, self.tok.sep_id
    res.pack = into
    if spans:
      res.src0 = buf('src0', n_pairs, torch.int64)
      res.src1 = buf('src1', n_pairs, torch.int64)
      _lib.check(L.lddl_row_spans(self.tok.handle, h, _ptr(res.src0), _ptr(res.src1), _ptr(res.tok_off),
                                  _ptr(res.len0), _ptr(res.len1), _ptr(res.flags), _ptr(res.bins),
                                  _ptr(res.part), _ptr(res.bin_count), s))
    else:
      _lib.check(L.lddl_materialize(self.tok.handle, h, _ptr(ids), _ptr(res.tokens), _ptr(res.tok_off),
                                    _ptr(res.len0), _ptr(res.len1), _ptr(res.flags), _ptr(res.bins),
                                    _ptr(res.part), _ptr(res.bin_count), s))
    res.bin_count = res.bin_count[:shards.n_part * nbins].view(shards.n_part, nbins)
    res.ids, res.ntok, res.ids_off = ids, ntok, tok_off
    if masking and not codebert:
      res.n_masked = int(tot[3])
      res.mlm_off = buf('mlm_off', n_pairs + 1, torch.int64)
      res.mlm_pos = buf('mlm_pos', res.n_masked, torch.int16)
      res.mlm_label = buf('mlm_label', res.n_masked, torch.int16)
      if spans:
        res.mlm_token = buf('mlm_token', res.n_masked, torch.int16)
        _lib.check(L.lddl_masked_lm_spans(self.tok.handle, h, _ptr(ids), _ptr(res.src0), _ptr(res.src1),
                                          _ptr(res.len0), _ptr(res.part), _ptr(res.mlm_off), _ptr(res.mlm_pos),
                                          _ptr(res.mlm_label), _ptr(res.mlm_token), s))
      else:
        _lib.check(L.lddl_masked_lm(self.tok.handle, h, _ptr(res.mlm_off), _ptr(res.mlm_pos), _ptr(res.mlm_label), s))
    return res

  def run(self, shards, **kw):
    return self.pack(shards, *self.tokenize(shards), **kw)

  def bin(self, num_tokens, bin_size, nbins, stream=None):
    return bin_rows(self.tok, num_tokens, bin_size, nbins, stream)


def bin_rows(tok, num_tokens, bin_size, nbins, stream=None):
  """lddl_bin: group rows by length bin as binning.py:63-93
  _to_dataframe_binned does.  num_tokens: int64 tensor on tok's device ->
  (perm, bin_counts) on the device: the row indices bin-major, ascending
  within a bin, and the rows per bin.  A length whose bin falls below -nbins
  raises IndexError, as the reference's seqs[bin_id] does."""
  if num_tokens.dtype != torch.int64 or not num_tokens.is_contiguous():
    raise ValueError('num_tokens: a contiguous int64 tensor')
  n = num_tokens.numel()
  perm = torch.empty(max(n, 1), dtype=torch.int64, device=num_tokens.device)
  counts = torch.empty(nbins, dtype=torch.int64, device=num_tokens.device)
  L = _lib.lib()
  rc = L.lddl_bin(tok.handle, _ptr(num_tokens), n, int(bin_size), int(nbins), _ptr(perm), _ptr(counts),
                  _stream(stream))
  if rc == -7:
    raise IndexError(L.lddl_last_error().decode())
  _lib.check(rc)
  return perm[:n], counts


def run_bert(corpus, vocab_file=VOCAB_BERT, target_seq_length=128, bin_size=None, n_partitions=1, seed=12345,
             device=None, check_host=False, duplicate_factor=5, short_seq_prob=0.1, part_doc_off=None,
             codebert=False, masking=False, masked_lm_ratio=0.15, spans=False):
  device = device or torch.device('cuda', 0)
  if part_doc_off is None:
    part_doc_off = partition_by_bytes(corpus, n_partitions)
  pk = Packer(vocab_file, device.index, masking=masking)
  sh = upload(corpus, part_doc_off, device)
  res = pk.run(sh, target_seq_length=target_seq_length, short_seq_prob=short_seq_prob,
               duplicate_factor=duplicate_factor, seed=seed, bin_size=bin_size, codebert=codebert,
               masking=masking, masked_lm_ratio=masked_lm_ratio, spans=spans)
  torch.cuda.synchronize(device)
  res.part_doc_off = np.asarray(part_doc_off)
  if check_host:
    res.ntok_host = res.ntok[:sh.n_sent].cpu().numpy()
  return res


def assert_same_pairs(res, expected):
  """expected: per partition, rows (A, B, is_random_next, num_tokens) in the
  reference's output order (oracle.pack_oracle.run_bert_shards)."""
  rows = res.rows()
  flat = [(p, r) for p, part in enumerate(expected) for r in part]
  assert len(rows) == len(flat), (len(rows), len(flat))
  for g, (row, (p, e)) in enumerate(zip(rows, flat)):
    pp, a, b, fl, bn, tok = row[:6]
    ea, eb, ern, en = e[:4]
    assert pp == p, ('partition', g, pp, p)
    assert a == list(ea) and b == list(eb), ('tokens', g)
    assert bool(fl & 1) == bool(ern), ('is_random_next', g)
    assert len(tok) == en, ('num_tokens', g)
    if len(e) > 4:  # masking: positions and labels
      assert row[6] == list(e[4]) and row[7] == list(e[5]), ('masked_lm', g)
