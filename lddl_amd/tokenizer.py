"""MI355X WordPiece tokenizer: drop-in for the BertTokenizerFast object the
reference builds in lddl/dask/bert/pretrain.py:584-587 and calls at :79-80.

``Tokenizer(vocab_file).tokenize(s, max_length=512, truncation=True)``
returns the same token strings (one sentence; convenience / parity surface),
``tokenize_device(...)`` is the batched hot-path entry: every sentence of a
shard in one launch, inputs and outputs resident in HBM.
"""
import ctypes

import numpy as np
import torch

from . import _lib

TOKENS_MAX = 65534  # lddl_tokenize's max_tok bound (u16 per-sentence counts)


def _ptr(t):
  return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(stream=None):
  s = stream if stream is not None else torch.cuda.current_stream()
  return ctypes.c_void_p(s.cuda_stream)


class CapacityError(RuntimeError):
  """lddl_tokenize's ids did not fit out_cap (LDDL_ECAPACITY): .total ids needed"""

  def __init__(self, total, cap):
    super().__init__('lddl_amd: %d token ids do not fit the %d-entry ids buffer' % (total, cap))
    self.total, self.cap = total, cap


class Tokenizer:
  """Owns the device vocab/Unicode tables for one GPU (one lddl_ctx)."""

  def __init__(self, vocab_file=_lib.VOCAB_BERT, device=None):
    if not torch.cuda.is_available():
      raise RuntimeError('lddl_amd.Tokenizer needs a ROCm GPU (no CPU fallback)')
    self.device = torch.device('cuda', torch.cuda.current_device() if device is None else device)
    L = _lib.lib()
    h = ctypes.c_void_p()
    _lib.check(L.lddl_create(vocab_file.encode(), _lib.TABLE_PATH.encode(), self.device.index,
                             ctypes.byref(h)))
    self._h = h
    self.vocab_file = vocab_file
    self.vocab_size = _lib.check(L.lddl_vocab_size(h))
    ids = (ctypes.c_int32 * 5)()
    _lib.check(L.lddl_special_ids(h, ids))
    self.pad_id, self.unk_id, self.cls_id, self.sep_id, self.mask_id = list(ids)
    with open(vocab_file, encoding='utf-8') as f:
      self.ids_to_tokens = [l.rstrip('\n').rstrip('\r') for l in f]
    if self.ids_to_tokens and self.ids_to_tokens[-1] == '' and len(self.ids_to_tokens) > self.vocab_size:
      self.ids_to_tokens.pop()
    self.vocab = {t: i for i, t in enumerate(self.ids_to_tokens)}

  def close(self):
    if getattr(self, '_h', None):
      _lib.lib().lddl_destroy(self._h)
      self._h = None

  def __del__(self):
    try:
      self.close()
    except Exception:
      pass

  @property
  def handle(self):
    return self._h

  # ---- batched hot path -------------------------------------------------
  def tokenize_device(self, data, sent_off, max_tok=512, out_ids=None, out_ntok=None, out_tok_off=None, stream=None,
                      nbytes=None):
    """data: uint8 cuda tensor; sent_off: int64 cuda tensor [n_sent+1].
    Returns the dense CSR result (ids, ntok, tok_off): ids int16 view of
    uint16, sentence s's ids at ids[tok_off[s]:tok_off[s+1]], ntok int32
    [n_sent] = their counts, tok_off int64 [n_sent+1].  nbytes = sent_off[-1]
    - sent_off[0] (default: data.numel(), i.e. data holds no padding).  The
    default ids buffer holds nbytes + 16 entries (#tokens <= #bytes, plus the
    16-entry pad lddl_materialize reads).  With a smaller out_ids the total
    tok_off[n_sent] is read back (one stream sync) and a total past its
    capacity raises (lddl_tokenize writes no id past out_cap): the caller
    grows the buffer and calls again (Packer.tokenize does)."""
    n_sent = sent_off.numel() - 1
    if nbytes is None:
      nbytes = int(data.numel())
    if out_ids is None:
      out_ids = torch.empty(max(nbytes, 1) + 16, dtype=torch.int16, device=self.device)
    if out_ntok is None:
      out_ntok = torch.empty(max(n_sent, 1), dtype=torch.int32, device=self.device)
    if out_tok_off is None:
      out_tok_off = torch.empty(n_sent + 1, dtype=torch.int64, device=self.device)
    assert data.dtype == torch.uint8 and sent_off.dtype == torch.int64
    assert data.is_cuda and sent_off.is_cuda and out_tok_off.numel() >= n_sent + 1
    cap = max(0, out_ids.numel() - 16)
    _lib.check(_lib.lib().lddl_tokenize(self._h, _ptr(data), nbytes, _ptr(sent_off), n_sent, max_tok,
                                        _ptr(out_ids), cap, _ptr(out_ntok), _ptr(out_tok_off), _stream(stream)))
    if cap < nbytes:
      total = self.total_tokens(out_tok_off, n_sent, stream)
      if total > cap:
        raise CapacityError(total, cap)
    return out_ids, out_ntok, out_tok_off

  @staticmethod
  def total_tokens(tok_off, n_sent, stream=None):
    """tok_off[n_sent] read back after the work queued on `stream`"""
    (stream if stream is not None else torch.cuda.current_stream()).synchronize()
    return int(tok_off[n_sent].item())

  def set_special_flags(self, on=True):
    """following tokenize calls record per-sentence [CLS]/[SEP] flags for a
    masked pack over the same buffers (lddl_set_special_flags)"""
    _lib.check(_lib.lib().lddl_set_special_flags(self.handle, 1 if on else 0))

  def set_algo(self, algo):
    """the tokenizer algorithm of the following calls (lddl_set_tokenize_algo:
    5 split, the default; 6 lane; 0 the exact serial path -- identical ids);
    returns the one selected (0 when the tables rule the asked one out)"""
    out = ctypes.c_int(-1)
    _lib.check(_lib.lib().lddl_set_tokenize_algo(self.handle, int(algo), ctypes.byref(out)))
    return out.value

  def set_timing(self, on=True):
    """per-kernel timing of the following tokenize calls (lddl_set_timing)"""
    _lib.check(_lib.lib().lddl_set_timing(self.handle, 1 if on else 0))

  def stats(self):
    """{'scan_ms', 'wordpiece_ms', 'expand_ms' (finish: serial-path tiles,
    counts, offset scan, dense expand; summed over the call's segments),
    'records', 'launches' (segments), 'fallback_tiles'} of the last call
    (synchronises on its events)"""
    out = (ctypes.c_double * 6)()
    _lib.check(_lib.lib().lddl_tokenize_stats(self.handle, out, 6))
    return {'scan_ms': out[0], 'wordpiece_ms': out[1], 'expand_ms': out[2], 'records': int(out[3]),
            'launches': int(out[4]), 'fallback_tiles': int(out[5])}

  def encode_batch(self, sentences, max_tok=512):
    """list[str] -> list[list[int]] (compact host result)."""
    enc = [s.encode('utf-8') for s in sentences]
    off = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum([len(b) for b in enc], out=off[1:])
    raw = np.frombuffer(b''.join(enc) + b'\0' * 16, dtype=np.uint8)
    d = torch.from_numpy(raw.copy()).to(self.device)
    o = torch.from_numpy(off).to(self.device)
    ids, ntok, toff = self.tokenize_device(d, o, max_tok)
    ids = ids.cpu().numpy().view(np.uint16)
    toff = toff.cpu().numpy()
    return [ids[toff[i]:toff[i + 1]].astype(np.int64).tolist() for i in range(len(enc))]

  # ---- reference-compatible surface --------------------------------------
  def tokenize(self, text, max_length=512, truncation=True, **kwargs):
    """Same result as BertTokenizerFast.tokenize as called at pretrain.py:79-80
    under transformers 4.16.2 (per-sentence truncation to max_length)."""
    cap = max_length if truncation else TOKENS_MAX
    ids = self.encode_batch([text], cap)[0]
    if not truncation and len(ids) >= TOKENS_MAX:
      # the device path counts tokens per sentence in 16 bits: a text this
      # long cannot be returned whole (BertTokenizerFast would)
      raise ValueError('lddl_amd: text reaches %d tokens; truncation=False cannot return it whole' % TOKENS_MAX)
    return [self.ids_to_tokens[i] for i in ids]

  def convert_tokens_to_ids(self, tokens):
    return [self.vocab.get(t, self.unk_id) for t in tokens]
