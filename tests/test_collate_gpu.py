"""GPU collate (lddl_collate_bert / lddl_mask_tokens via lddl_amd.loader)
against the reference's _to_encoded_inputs outputs (golden) and the oracle;
dynamic masking against _mask_tokens' distribution (bert.py:156-196).

Tolerances of the statistical test (dynamic masking; the reference draws
from torch's CPU generator, this from a counter-based hash): on ~200 k
candidate columns, the mask rate is within 0.005 of mlm_probability and the
[MASK] / random / kept split within 0.015 of 0.8 / 0.1 / 0.1 (> 6 sigma)."""
import io

import numpy as np
import pytest
import torch

from lddl_amd import _lib
from oracle.collate_oracle import CollateOracle
from test_collate_oracle import CASES, VOCABS, case_batch

pytestmark = pytest.mark.gpu

_COLL = {}


def collate(gpu, vocab='bert', **kw):
  from lddl_amd.loader import BertCollate
  key = (vocab, tuple(sorted(kw.items())))
  if key not in _COLL:
    _COLL[key] = BertCollate(VOCABS[vocab], device=0, **kw)
  return _COLL[key]


def _np(t):
  return t.cpu().numpy()


@pytest.mark.parametrize('k', range(len(CASES)))
def test_collate_matches_reference_golden(gpu, k):
  c = CASES[k]
  col = collate(gpu, c['vocab'], sequence_length_alignment=c['align'], ignore_index=c['ignore_index'])
  out = col.to_encoded_inputs(case_batch(c))
  keys = ['input_ids', 'token_type_ids', 'attention_mask', 'next_sentence_labels',
          'labels' if c['static'] else 'special_tokens_mask']
  for key in keys:
    assert np.array_equal(_np(out[key]), np.asarray(c[key], np.int64)), key


def _random_batch(rng, vocab, n, max_len, static):
  V = vocab
  out = []
  for _ in range(n):
    na = int(rng.integers(0, max_len))
    nb = int(rng.integers(0, max(1, max_len - na)))
    ta = [V[int(i)] for i in rng.integers(0, len(V), na)]
    tb = [V[int(i)] for i in rng.integers(0, len(V), nb)]
    rn = bool(rng.random() < 0.5)
    if not static:
      out.append((' '.join(ta), ' '.join(tb), rn))
      continue
    nt = na + nb + 3
    cand = [i for i in range(1, nt - 1) if i != na + 1]
    k = min(len(cand), max(1, round(nt * 0.15)))
    pos = np.sort(rng.choice(cand, k, replace=False)).astype(np.uint16) if cand else np.zeros(0, np.uint16)
    bio = io.BytesIO()
    np.save(bio, pos)
    lab = ' '.join(V[int(i)] for i in rng.integers(0, len(V), len(pos)))
    out.append((' '.join(ta), ' '.join(tb), rn, bio.getvalue(), lab))
  return out


def _vocab(path):
  with open(path, encoding='utf-8') as f:
    return [l.rstrip('\n') for l in f]


@pytest.mark.parametrize('static', [False, True])
def test_collate_matches_oracle_large(gpu, static):
  V = _vocab(_lib.VOCAB_BERT)
  rng = np.random.default_rng(5)
  batch = _random_batch(rng, V, 256, 509, static)
  out = collate(gpu).to_encoded_inputs(batch)
  exp = CollateOracle(_lib.VOCAB_BERT).encode(batch)
  for key, v in exp.items():
    assert np.array_equal(_np(out[key]), v), key


def test_collate_arrow_path_matches_list_path(gpu, tmp_path):
  import pyarrow as pa
  import pyarrow.parquet as pq
  V = _vocab(_lib.VOCAB_BERT)
  batch = _random_batch(np.random.default_rng(9), V, 64, 128, True)
  t = pa.table({'A': [b[0] for b in batch], 'B': [b[1] for b in batch],
                'is_random_next': [b[2] for b in batch],
                'num_tokens': pa.array([len(b[0].split()) + len(b[1].split()) + 3 for b in batch], pa.uint16()),
                'masked_lm_positions': pa.array([b[3] for b in batch], pa.binary()),
                'masked_lm_labels': [b[4] for b in batch]})
  pq.write_table(t, str(tmp_path / 'part.0.parquet'))
  rt = pq.read_table(str(tmp_path / 'part.0.parquet'))
  col = collate(gpu)
  a = col.collate_arrow(rt.slice(7, 40))  # non-zero array offset
  b = col(batch[7:47])
  for key in a:
    assert torch.equal(a[key], b[key]), key


def test_dynamic_fused_equals_two_step(gpu):
  from lddl_amd.loader import BertCollate
  V = _vocab(_lib.VOCAB_BERT)
  batch = _random_batch(np.random.default_rng(3), V, 128, 300, False)
  c1 = BertCollate(_lib.VOCAB_BERT, device=0, base_seed=77)
  c2 = BertCollate(_lib.VOCAB_BERT, device=0, base_seed=77)
  fused = c1(batch)
  enc = c2.to_encoded_inputs(batch)
  ids, labels = c2.mask_tokens(enc['input_ids'].clone(), enc['special_tokens_mask'], counter=0)
  assert torch.equal(fused['input_ids'], ids)
  assert torch.equal(fused['labels'], labels)
  # a second batch draws different masks
  again = c1(batch)
  assert not torch.equal(again['labels'], fused['labels'])


def test_dynamic_masking_statistics(gpu):
  from lddl_amd.loader import BertCollate
  V = _vocab(_lib.VOCAB_BERT)
  batch = _random_batch(np.random.default_rng(11), V, 512, 509, False)
  col = BertCollate(_lib.VOCAB_BERT, device=0, base_seed=2024, mlm_probability=0.15, ignore_index=-1)
  enc = col.to_encoded_inputs(batch)
  orig = _np(enc['input_ids'])
  sp = _np(enc['special_tokens_mask']).astype(bool)
  out = col(batch)
  ids, lab = _np(out['input_ids']), _np(out['labels'])
  masked = lab != -1
  assert not (masked & sp).any()  # specials and padding never selected
  assert np.array_equal(lab[masked], orig[masked])  # labels = original ids
  assert np.array_equal(ids[~masked], orig[~masked])
  cand = int((~sp).sum())
  rate = masked.sum() / cand
  assert abs(rate - 0.15) < 0.005, rate
  m = ids[masked]
  o = orig[masked]
  frac_mask = np.mean(m == 103)
  frac_keep = np.mean((m == o) & (m != 103))
  frac_rand = 1 - frac_mask - frac_keep
  assert abs(frac_mask - 0.8) < 0.015 and abs(frac_keep - 0.1) < 0.015 and abs(frac_rand - 0.1) < 0.015
  assert ids.max() < col.tok.vocab_size and ids.min() >= 0
  for key in ('token_type_ids', 'attention_mask', 'next_sentence_labels'):
    assert torch.equal(out[key], enc[key])


def test_mlm_probability_edges(gpu):
  from lddl_amd.loader import BertCollate
  V = _vocab(_lib.VOCAB_BERT)
  batch = _random_batch(np.random.default_rng(2), V, 32, 100, False)
  z = BertCollate(_lib.VOCAB_BERT, device=0, mlm_probability=0.0)(batch)
  assert bool((z['labels'] == -1).all())
  one = BertCollate(_lib.VOCAB_BERT, device=0, mlm_probability=1.0)
  enc = one.to_encoded_inputs(batch)
  full = one(batch)
  assert torch.equal(full['labels'] != -1, enc['special_tokens_mask'] == 0)


def test_errors(gpu):
  from lddl_amd.loader import BertCollate
  col = BertCollate(_lib.VOCAB_BERT, device=0)
  bio = io.BytesIO()
  np.save(bio, np.asarray([40], np.uint16))  # position past the padded row
  with pytest.raises(IndexError):
    col([('hello world', 'the', True, bio.getvalue(), 'hello')])
  with pytest.raises(RuntimeError):  # positions / labels count mismatch
    col([('hello world', 'the', True, bio.getvalue(), 'hello world')])
  with pytest.raises(RuntimeError):  # not np.save bytes
    col([('hello world', 'the', True, b'garbage!', 'hello')])
  with pytest.raises(RuntimeError):  # longer than the 2048-column LDS row
    col([(' '.join(['the'] * 2100), '', False)])
  with pytest.raises(ValueError):
    col.collate_arrow.__self__._run([], np.zeros(0, np.uint8), False)
