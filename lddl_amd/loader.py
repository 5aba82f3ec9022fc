"""Training-time collate of LDDL parquet rows on the GPU.

Drop-in for the collate the reference installs in
``get_bert_pretrain_data_loader`` (lddl/torch/bert.py:354-371
``_batch_preprocess``): ``_to_encoded_inputs`` (bert.py:69-153) turns a batch
of samples ``(A, B, is_random_next[, masked_lm_positions, masked_lm_labels])``
into padded int64 tensors, and ``_mask_tokens`` (bert.py:156-196) applies the
dynamic 80/10/10 masking when the shards carry no static masks.  Here both are
one HIP kernel (``lddl_collate_bert``, csrc/collate.hip): the batch's string
columns are staged in one pinned buffer, copied once, split / looked up /
padded / masked on the device, and the outputs stay in HBM for the model.

Differences from the reference, by design:
* dynamic masking draws from a counter-based hash of (seed, batch counter, row,
  column), not torch's CPU generator: the same distribution (mask rate
  ``mlm_probability``, 80 % [MASK] / 10 % random / 10 % kept), not the same
  stream;
* outputs are CUDA tensors (the reference returns CPU tensors that the
  training loop moves with ``.to(device)``).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .tokenizer import Tokenizer, _stream

MODE_SPECIAL_MASK, MODE_STATIC, MODE_DYNAMIC = 0, 1, 2


def _column(values, encode):
  """list of str/bytes -> (uint8 bytes, int64 offsets)"""
  enc = [v.encode('utf-8') for v in values] if encode else [bytes(v) for v in values]
  off = np.zeros(len(enc) + 1, dtype=np.int64)
  if enc:
    np.cumsum([len(b) for b in enc], out=off[1:])
  return np.frombuffer(b''.join(enc), dtype=np.uint8), off


def _arrow_column(arr):
  """pa.StringArray / BinaryArray (or a ChunkedArray) -> (uint8 bytes, int64
  offsets), zero-copy on the bytes"""
  import pyarrow as pa
  if isinstance(arr, pa.ChunkedArray):
    arr = arr.combine_chunks()
  if pa.types.is_large_string(arr.type) or pa.types.is_large_binary(arr.type):
    odt = np.int64
  else:
    odt = np.int32
  bufs = arr.buffers()
  off = np.frombuffer(bufs[1], dtype=odt)[arr.offset:arr.offset + len(arr) + 1].astype(np.int64)
  data = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None else np.zeros(0, np.uint8)
  return data, off


class BertCollate:
  """``collate(batch) -> dict`` with the keys of bert.py:129-152 plus
  ``labels`` (masked): input_ids, token_type_ids, attention_mask, labels,
  next_sentence_labels -- int64 tensors on the GPU.

  batch: a list of samples as the reference's DataLoader hands to its
  collate_fn (tuples of 3 or 5 fields), or a pyarrow RecordBatch / Table of
  the shard schema (zero-copy columns; ``collate_arrow``)."""

  def __init__(self, vocab_file=_lib.VOCAB_BERT, device=None, sequence_length_alignment=8, ignore_index=-1,
               mlm_probability=0.15, base_seed=12345, tokenizer=None):
    assert isinstance(sequence_length_alignment, int) and sequence_length_alignment >= 1
    assert isinstance(mlm_probability, (int, float)) and 0 <= mlm_probability <= 1
    self.tok = tokenizer if tokenizer is not None else Tokenizer(vocab_file, device)
    self.device = self.tok.device
    self.sequence_length_alignment = sequence_length_alignment
    self.ignore_index = int(ignore_index)
    self.mlm_probability = float(mlm_probability)
    self.seed = int(base_seed) & ((1 << 64) - 1)
    self.counter = 0  # one per collated batch: the dynamic masks differ per batch

  # ---- staging ------------------------------------------------------------
  def _upload(self, cols, is_random_next):
    """One pinned host buffer holding every column (16-B aligned pieces), one
    H2D copy; returns device addresses of each piece."""
    pieces = []
    for data, off in cols:
      pieces.append(data)
      pieces.append(off.view(np.uint8))
    pieces.append(np.ascontiguousarray(is_random_next, dtype=np.uint8))
    starts, pos = [], 0
    for p in pieces:
      starts.append(pos)
      pos += (p.nbytes + 15) & ~15
    host = torch.empty(max(pos, 16), dtype=torch.uint8, pin_memory=True)
    hn = host.numpy()
    for p, s in zip(pieces, starts):
      hn[s:s + p.nbytes] = p
    dev = torch.empty_like(host, device=self.device)
    dev.copy_(host, non_blocking=True)
    base = dev.data_ptr()
    return dev, host, [base + s for s in starts]

  def _run(self, cols, is_random_next, static):
    L = _lib.lib()
    n = len(is_random_next)
    if n == 0:
      raise ValueError('empty batch')  # max() of an empty sequence in bert.py:94-95
    dev, host, ptrs = self._upload(cols, is_random_next)
    st = _stream()
    P = ctypes.c_void_p
    seq = ctypes.c_int64()
    _lib.check(L.lddl_collate_seq_len(self.tok.handle, P(ptrs[0]), P(ptrs[1]), P(ptrs[2]), P(ptrs[3]), n,
                                      self.sequence_length_alignment, ctypes.byref(seq), st))
    S = int(seq.value)
    out = torch.empty((5, n, S), dtype=torch.int64, device=self.device)
    nsl = torch.empty(n, dtype=torch.int64, device=self.device)
    if static:
      pos_d, pos_o, lab_d, lab_o = ptrs[4:8]
    else:
      pos_d = pos_o = lab_d = lab_o = 0
    mode = MODE_STATIC if static else MODE_DYNAMIC
    rc = L.lddl_collate_bert(self.tok.handle, P(ptrs[0]), P(ptrs[1]), P(ptrs[2]), P(ptrs[3]), P(ptrs[-1]),
                             P(pos_d), P(pos_o), P(lab_d), P(lab_o), n, S, mode, self.ignore_index,
                             self.mlm_probability, self.seed, self.counter, P(out[0].data_ptr()),
                             P(out[1].data_ptr()), P(out[2].data_ptr()), P(out[3].data_ptr()), P(nsl.data_ptr()), st)
    self.counter += 1
    if rc == -7:
      raise IndexError(L.lddl_last_error().decode())
    _lib.check(rc)
    del dev, host  # the stream was synchronised by the call
    return {'input_ids': out[0], 'token_type_ids': out[1], 'attention_mask': out[2],
            'next_sentence_labels': nsl, 'labels': out[3]}

  # ---- entry points ---------------------------------------------------------
  def __call__(self, batch):
    if hasattr(batch, 'schema'):
      return self.collate_arrow(batch)
    static = len(batch[0]) > 3
    if static:
      assert len(batch[0]) == 5
    cols = [_column([s[0] for s in batch], True), _column([s[1] for s in batch], True)]
    if static:
      cols.append(_column([s[3] for s in batch], False))
      cols.append(_column([s[4] for s in batch], True))
    rn = np.fromiter((bool(s[2]) for s in batch), dtype=np.uint8, count=len(batch))
    return self._run(cols, rn, static)

  def collate_arrow(self, table):
    """A pyarrow RecordBatch/Table with the shard schema (pretrain.py:457-471)."""
    names = table.schema.names
    static = 'masked_lm_positions' in names
    if static:
      assert 'masked_lm_labels' in names
    cols = [_arrow_column(table.column('A')), _arrow_column(table.column('B'))]
    if static:
      cols.append(_arrow_column(table.column('masked_lm_positions')))
      cols.append(_arrow_column(table.column('masked_lm_labels')))
    rn = np.asarray(table.column('is_random_next').to_numpy(zero_copy_only=False), dtype=np.uint8)
    return self._run(cols, rn, static)

  # ---- the reference's two steps, separately ----------------------------------
  def to_encoded_inputs(self, batch):
    """bert.py:69-153 as is: with static masks 'labels', else
    'special_tokens_mask' (dynamic masking left to mask_tokens)."""
    static = len(batch[0]) > 3
    if static:
      return self(batch)
    L = _lib.lib()
    n = len(batch)
    cols = [_column([s[0] for s in batch], True), _column([s[1] for s in batch], True)]
    rn = np.fromiter((bool(s[2]) for s in batch), dtype=np.uint8, count=n)
    dev, host, ptrs = self._upload(cols, rn)
    st = _stream()
    P = ctypes.c_void_p
    seq = ctypes.c_int64()
    _lib.check(L.lddl_collate_seq_len(self.tok.handle, P(ptrs[0]), P(ptrs[1]), P(ptrs[2]), P(ptrs[3]), n,
                                      self.sequence_length_alignment, ctypes.byref(seq), st))
    S = int(seq.value)
    out = torch.empty((4, n, S), dtype=torch.int64, device=self.device)
    nsl = torch.empty(n, dtype=torch.int64, device=self.device)
    _lib.check(L.lddl_collate_bert(self.tok.handle, P(ptrs[0]), P(ptrs[1]), P(ptrs[2]), P(ptrs[3]), P(ptrs[-1]),
                                   P(0), P(0), P(0), P(0), n, S, MODE_SPECIAL_MASK, self.ignore_index,
                                   self.mlm_probability, self.seed, self.counter, P(out[0].data_ptr()),
                                   P(out[1].data_ptr()), P(out[2].data_ptr()), P(out[3].data_ptr()),
                                   P(nsl.data_ptr()), st))
    del dev, host
    return {'input_ids': out[0], 'token_type_ids': out[1], 'attention_mask': out[2],
            'next_sentence_labels': nsl, 'special_tokens_mask': out[3]}

  def mask_tokens(self, inputs, special_tokens_mask, counter=None):
    """bert.py:156-196 on device tensors: masks ``inputs`` in place and
    returns (inputs, labels).  counter: the batch counter of the draws
    (default: the next one)."""
    assert inputs.dtype == torch.int64 and inputs.is_cuda and inputs.is_contiguous()
    sp = special_tokens_mask.to(device=self.device, dtype=torch.int64).contiguous()
    assert sp.shape == inputs.shape
    labels = torch.empty_like(inputs)
    n, S = inputs.shape
    if counter is None:
      counter = self.counter
      self.counter += 1
    _lib.check(_lib.lib().lddl_mask_tokens(self.tok.handle, ctypes.c_void_p(inputs.data_ptr()),
                                           ctypes.c_void_p(sp.data_ptr()), ctypes.c_void_p(labels.data_ptr()), n,
                                           S, self.mlm_probability, self.ignore_index, self.seed, counter,
                                           _stream()))
    return inputs, labels
