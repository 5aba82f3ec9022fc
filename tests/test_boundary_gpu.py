"""The C-ABI's pack-result handle (lddl_pack_new / lddl_pack_free: post-pack
calls name the result they read) and the standalone binning entry point
lddl_bin (binning.py:63-93 _to_dataframe_binned), called through the C-ABI
and checked against oracle/pack_oracle.py (binned_order, the restatement of
binning.py:70-75) and against the packer's own binned rows."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import pack_oracle as po

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def packer(gpu):
  from lddl_amd.pipeline import Packer, VOCAB_BERT
  return Packer(VOCAB_BERT, 0)


def _bin(packer, nt, bin_size, nbins):
  from lddl_amd.pipeline import bin_rows
  t = torch.from_numpy(np.ascontiguousarray(nt, dtype=np.int64)).cuda()
  perm, cnt = bin_rows(packer.tok, t, bin_size, nbins)
  return perm.cpu().numpy(), cnt.cpu().numpy()


def _stable_bins(nt, bin_size, nbins):
  """vectorised binned_order for large n: the bin of every row (Python
  floor division, capped, negative bins from the end), then a stable sort"""
  b = np.floor_divide(nt.astype(np.int64) - 1, bin_size)
  b = np.minimum(b, nbins - 1)
  b = np.where(b < 0, b + nbins, b)
  return np.argsort(b, kind='stable'), np.bincount(b, minlength=nbins)


@pytest.mark.parametrize('n', [0, 1, 63, 64, 65, 4095, 4096, 4097, 20_011])
@pytest.mark.parametrize('bin_size,nbins', [(32, 4), (64, 8), (1, 1), (16, 1024), (7, 3)])
def test_lddl_bin_vs_oracle(packer, n, bin_size, nbins):
  rng = np.random.default_rng(n * 31 + nbins)
  nt = rng.integers(-bin_size * (nbins - 1), bin_size * nbins + 40, size=n)
  nt[rng.random(n) < 0.05] = 0  # length 0 -> bin -1 -> the last bin
  perm, cnt = _bin(packer, nt, bin_size, nbins)
  order, counts = po.binned_order(nt.tolist(), bin_size, nbins)
  assert perm.tolist() == order
  assert cnt.tolist() == counts


@pytest.mark.parametrize('dist', ['uniform', 'one_bin', 'sorted_desc'])
def test_lddl_bin_large(packer, dist):
  """5M rows (1221 wave chunks): bit-exact against a stable sort of the
  reference's bin ids"""
  rng = np.random.default_rng(3)
  n = 5_000_000
  if dist == 'uniform':
    nt = rng.integers(1, 513, size=n)
  elif dist == 'one_bin':
    nt = np.full(n, 100)
  else:
    nt = np.sort(rng.integers(0, 600, size=n))[::-1].copy()
  perm, cnt = _bin(packer, nt, 64, 8)
  order, counts = _stable_bins(nt, 64, 8)
  assert np.array_equal(perm, order)
  assert np.array_equal(cnt, counts)


def test_lddl_bin_index_error(packer):
  """a bin below -nbins: the reference's seqs[bin_id] raises IndexError"""
  nt = np.array([5, 3, -200, 7], dtype=np.int64)
  with pytest.raises(IndexError):
    _bin(packer, nt, 32, 4)
  # in range negative bins index from the end (bin -2 -> nbins - 2)
  perm, cnt = _bin(packer, np.array([5, -40, 0, 200]), 32, 4)
  assert perm.tolist() == po.binned_order([5, -40, 0, 200], 32, 4)[0]
  assert cnt.tolist() == [1, 0, 1, 2]


def test_lddl_bin_bad_args(packer):
  from lddl_amd import _lib
  L = _lib.lib()
  h = packer.tok.handle
  x = torch.zeros(4, dtype=torch.int64, device='cuda')
  y = torch.zeros(4, dtype=torch.int64, device='cuda')
  p = ctypes.c_void_p
  s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
  assert L.lddl_bin(h, p(x.data_ptr()), 4, 0, 4, p(y.data_ptr()), p(y.data_ptr()), s) == -1
  assert L.lddl_bin(h, p(x.data_ptr()), 4, 32, 0, p(y.data_ptr()), p(y.data_ptr()), s) == -1
  assert L.lddl_bin(h, p(x.data_ptr()), 4, 32, 1025, p(y.data_ptr()), p(y.data_ptr()), s) == -1
  assert L.lddl_bin(h, p(x.data_ptr()), 4, 32, 4, None, p(y.data_ptr()), s) == -1


def test_lddl_bin_equals_pack_binning(packer):
  """binning a partition's unbinned (shuffled) rows with lddl_bin gives the
  packer's binned rows: the same grouping, applied after the same shuffle
  (pretrain.py:396-402 then binning.py:63-93)"""
  from lddl_amd import synth, pipeline
  c = synth.make_wiki(400_000, seed=21)
  pdo = pipeline.partition_by_bytes(c, 3)
  sh = pipeline.upload(c, pdo, 'cuda')
  ids, ntok, toff = packer.tokenize(sh)
  kw = dict(target_seq_length=128, seed=77, duplicate_factor=2)
  u = packer.pack(sh, ids, ntok, toff, **kw)
  urows = u.rows()
  b = packer.pack(sh, ids, ntok, toff, bin_size=32, **kw)
  brows = b.rows()
  assert len(urows) == len(brows) > 0
  got = []
  for p in range(3):
    part = [r for r in urows if r[0] == p]
    nt = np.array([len(r[5]) for r in part], dtype=np.int64)
    perm, cnt = _bin(packer, nt, 32, 4)
    assert np.array_equal(cnt, b.bin_count[p].cpu().numpy())
    got += [part[i][:4] + (int(np.searchsorted(np.cumsum(cnt), k, side='right')),) + part[i][5:]
            for k, i in enumerate(perm)]
  assert got == brows


# ------------------------------------------------------- pack results ----

def _raw_pack(packer, h, sh, ntok, toff, seq, bin_size, seed):
  from lddl_amd import _lib
  from lddl_amd.tokenizer import _ptr, _stream
  tot = (ctypes.c_int64 * 4)()
  rc = _lib.lib().lddl_pack_bert(packer.tok.handle, h, None, _ptr(ntok), _ptr(toff), _ptr(sh.sent_off), sh.n_sent,
                                 _ptr(sh.doc_sent_off), sh.n_doc, _ptr(sh.part_doc_off), sh.n_part, seq, 0.1, 2, 0,
                                 0.15, seed, bin_size, tot, _stream())
  return rc, [int(v) for v in tot]


def _raw_rows(packer, h, ids, tot, n_part):
  """lddl_materialize + lddl_row_docs of pack result h -> host arrays"""
  from lddl_amd import _lib
  from lddl_amd.tokenizer import _ptr, _stream
  L = _lib.lib()
  n, ntk, nb = tot[0], tot[1], tot[2]
  dev = 'cuda'
  tokens = torch.empty(ntk + 16, dtype=torch.int16, device=dev)
  off = torch.empty(n + 1, dtype=torch.int64, device=dev)
  l0, l1 = (torch.empty(max(n, 1), dtype=torch.int16, device=dev) for _ in range(2))
  fl, bn = (torch.empty(max(n, 1), dtype=torch.uint8, device=dev) for _ in range(2))
  part = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
  bc = torch.empty(n_part * nb, dtype=torch.int64, device=dev)
  docs = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
  _lib.check(L.lddl_materialize(packer.tok.handle, h, _ptr(ids), _ptr(tokens), _ptr(off), _ptr(l0), _ptr(l1),
                                _ptr(fl), _ptr(bn), _ptr(part), _ptr(bc), _stream()))
  _lib.check(L.lddl_row_docs(packer.tok.handle, h, _ptr(docs), _stream()))
  torch.cuda.synchronize()
  return [t.cpu().numpy() for t in (tokens[:ntk], off, l0[:n], l1[:n], fl[:n], bn[:n], part[:n], bc, docs[:n])]


def test_two_pack_results_coexist(packer):
  """two shard sets packed into two lddl_pack results back to back, then
  both materialised: each equals the same pack done alone through the ctx's
  own result (NULL)"""
  from lddl_amd import synth, pipeline
  cs = [synth.make_wiki(300_000, seed=5), synth.make_wiki(200_000, seed=6)]
  cfg = [(128, 32, 11), (256, 64, 12)]
  sets = []
  for c in cs:
    sh = pipeline.upload(c, pipeline.partition_by_bytes(c, 2), 'cuda')
    ids, ntok, toff = packer.tokenize(sh)
    sets.append((sh, ids.clone(), ntok.clone(), toff.clone()))
  alone = []
  for (sh, ids, ntok, toff), (seq, bs, seed) in zip(sets, cfg):
    rc, tot = _raw_pack(packer, None, sh, ntok, toff, seq, bs, seed)
    assert rc == 0 and tot[0] > 0
    alone.append((tot, _raw_rows(packer, None, ids, tot, 2)))
  hs = [pipeline.PackHandle(packer.tok) for _ in range(2)]
  assert hs[0].rows() == -1
  tots = []
  for h, (sh, ids, ntok, toff), (seq, bs, seed) in zip(hs, sets, cfg):
    rc, tot = _raw_pack(packer, h.handle, sh, ntok, toff, seq, bs, seed)
    assert rc == 0
    tots.append(tot)
  for k in (1, 0):  # the older result read last
    assert tots[k] == alone[k][0] and hs[k].rows() == tots[k][0]
    got = _raw_rows(packer, hs[k].handle, sets[k][1], tots[k], 2)
    for a, b in zip(got, alone[k][1]):
      assert np.array_equal(a, b)
  for h in hs:
    h.close()


def test_packer_results_into_two_handles_stay_live(packer):
  """Packer.pack into a second PackHandle keeps its PackResult
  columns in buffers of that handle, so the first result's columns are not
  overwritten (each equals the same pack done alone)"""
  from lddl_amd import synth, pipeline
  cs = [synth.make_wiki(300_000, seed=15), synth.make_wiki(250_000, seed=16)]
  cfg = [dict(target_seq_length=128, bin_size=32, seed=3), dict(target_seq_length=256, bin_size=64, seed=4)]
  sets = []
  for c in cs:
    sh = pipeline.upload(c, pipeline.partition_by_bytes(c, 2), 'cuda')
    ids, ntok, toff = packer.tokenize(sh)
    sets.append((sh, ids.clone(), ntok.clone(), toff.clone()))
  alone = [packer.pack(sh, ids, ntok, toff, spans=True, **kw).rows() for (sh, ids, ntok, toff), kw in zip(sets, cfg)]
  h2 = pipeline.PackHandle(packer.tok)
  try:
    r1 = packer.pack(*sets[0], spans=True, **cfg[0])
    r2 = packer.pack(*sets[1], spans=True, into=h2, **cfg[1])
    assert r2.rows() == alone[1]
    assert r1.rows() == alone[0]  # (read after the second pack)
  finally:
    h2.close()


def test_pack_result_states(packer):
  """a fresh result has nothing to materialise; a failed pack empties the
  result it was packing into and leaves the others alone"""
  from lddl_amd import _lib, synth, pipeline
  L = _lib.lib()
  h = pipeline.PackHandle(packer.tok)
  x = torch.zeros(64, dtype=torch.int64, device='cuda')
  assert L.lddl_row_docs(packer.tok.handle, h.handle, ctypes.c_void_p(x.data_ptr()), None) == -1
  c = synth.make_wiki(100_000, seed=9)
  sh = pipeline.upload(c, pipeline.partition_by_bytes(c, 1), 'cuda')
  ids, ntok, toff = packer.tokenize(sh)
  other = pipeline.PackHandle(packer.tok)
  assert _raw_pack(packer, other.handle, sh, ntok, toff, 128, 32, 1)[0] == 0
  assert _raw_pack(packer, h.handle, sh, ntok, toff, 128, 32, 1)[0] == 0
  assert h.rows() > 0
  rc, _ = _raw_pack(packer, h.handle, sh, ntok, toff, 128, 48, 1)  # 48 does not divide 128: EINVAL
  assert rc == -1
  assert h.rows() > 0  # argument errors are rejected before the result is touched
  # a pack that fails on the data (AssertionError of pretrain.py:330-331 needs a
  # crafted corpus) is covered by the pack tests; here: the other result is intact
  assert other.rows() > 0
  h.close()
  other.close()
