"""The Python packer restatement (oracle/pack_oracle.py) against golden rows
produced by the reference's own create_pairs_from_document
(tools/gen_golden_pack.py).  CPU only."""
import gzip
import json
import os

import pytest

from conftest import GOLDEN
from oracle import pack_oracle as po


def load(name):
  with gzip.open(os.path.join(GOLDEN, name), 'rt') as f:
    return json.load(f)


BERT = load('pack_bert.json.gz')
CODE = load('pack_codebert.json.gz')


def bert_rows(case):
  c = case['cfg']
  docs = [[s for s in d if s] for d in case['docs']]
  docs = [d for d in docs if d]
  pairs = po.partition_pairs(docs, case['seed'],
                             lambda D, di, r: po.bert_pairs(D, di, c['max_seq'], c['ssp'], r), c['dup'])
  return docs, pairs


@pytest.mark.parametrize('k', [i for i, c in enumerate(BERT['cases']) if not c['cfg']['masking']])
def test_bert_pairs_match_reference(k):
  case = BERT['cases'][k]
  if case['error']:
    with pytest.raises(AssertionError):
      bert_rows(case)
    return
  docs, pairs = bert_rows(case)
  rows = case['rows']
  assert len(pairs) == len(rows)
  for pr, row in zip(pairs, rows):
    a, b, rn = po.pair_tokens(docs, pr)
    assert (a, b, rn, len(a) + len(b) + 3) == (row['A'], row['B'], row['is_random_next'], row['num_tokens'])
  assert [po.bin_of(r['num_tokens'], case['bin_size'], case['nbins']) for r in rows] == case['bins']


@pytest.mark.parametrize('k', range(len(CODE['cases'])))
def test_codebert_pairs_match_reference(k):
  case = CODE['cases'][k]
  c = case['cfg']
  docs, nd = [], []
  for d, n in zip(case['docs'], case['ndoc']):
    ds = [s for s in d[:n] if s]
    cs = [s for s in d[n:] if s]
    if cs:
      docs.append(ds + cs)
      nd.append(len(ds))

  def run():
    return po.partition_pairs(docs, case['seed'],
                              lambda D, di, r: po.codebert_pairs(D, nd, di, c['max_seq'], c['ssp'], r), c['dup'])
  if case['error']:
    with pytest.raises(IndexError):
      run()
    return
  pairs = run()
  assert len(pairs) == len(case['rows'])
  for (doc_s, code_s, dw, cw), row in zip(pairs, case['rows']):
    dt = [t for (d, s) in doc_s for t in docs[d][s]][dw[0]:dw[1]]
    ct = [t for (d, s) in code_s for t in docs[d][s]][cw[0]:cw[1]]
    special = 3 if nd[code_s[0][0]] else 2
    assert (dt, ct, len(dt) + len(ct) + special) == (row['doc'], row['code'], row['num_tokens'])


BERT_MASK = (0.15, 30522, 101, 102, 103)  # ratio, |vocab|, [CLS], [SEP], [MASK]


@pytest.mark.parametrize('k', [i for i, c in enumerate(BERT['cases']) if c['cfg']['masking']])
def test_bert_masked_pairs_match_reference(k):
  """Static masking (pretrain.py:182-238) on the reference's own rows."""
  case = BERT['cases'][k]
  c = case['cfg']
  docs = [[s for s in d if s] for d in case['docs']]
  docs = [d for d in docs if d]
  if case['error']:
    with pytest.raises(AssertionError):
      po.partition_pairs(docs, case['seed'],
                         lambda D, di, r: po.bert_pairs(D, di, c['max_seq'], c['ssp'], r, BERT_MASK), c['dup'])
    return
  pairs = po.partition_pairs(docs, case['seed'],
                             lambda D, di, r: po.bert_pairs(D, di, c['max_seq'], c['ssp'], r, BERT_MASK), c['dup'])
  rows = case['rows']
  assert len(pairs) == len(rows)
  n_masked = 0
  for pr, row in zip(pairs, rows):
    a, b, rn = po.pair_tokens(docs, pr)
    ma, mb, pos, lab = pr[5]
    assert (ma, mb, rn, len(a) + len(b) + 3) == (row['A'], row['B'], row['is_random_next'], row['num_tokens'])
    assert pos == row['masked_lm_positions'] and lab == row['masked_lm_labels']
    n_masked += len(pos)
  assert n_masked > 0 or not rows
