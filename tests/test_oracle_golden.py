"""The oracle (C restatement of HF tokenizers) against the committed golden
vectors produced by tokenizers 0.22.2 (tools/gen_golden_tokenizer.py,
tools/gen_unicode_table.py).  CPU only."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from oracle.oracle import OracleTokenizer, compact

VOCABS = {'bert': os.path.join(ROOT, 'lddl_amd', 'data', 'bert_vocab.txt'),
          'codebert': os.path.join(ROOT, 'lddl_amd', 'data', 'codebert_52000_vocab.txt')}


@pytest.mark.parametrize('name', ['bert', 'codebert'])
def test_oracle_tokenizer_matches_golden(golden, name):
  g = golden('tok_%s.npz' % name)
  tok = OracleTokenizer(VOCABS[name])
  ids, ntok = tok.run(g['data'], g['sent_off'], 512, nthreads=4)
  assert np.array_equal(ntok, g['ntok'])
  exp = np.split(g['ids'], np.cumsum(g['ntok'])[:-1])
  got = compact(ids, ntok, g['sent_off'])
  bad = [i for i, (a, b) in enumerate(zip(exp, got)) if not np.array_equal(a, b)]
  assert not bad, bad[:10]


def test_oracle_normalizer_fuzz():
  d = json.load(open(os.path.join(GOLDEN, 'normalize_fuzz.json')))
  tok = OracleTokenizer(VOCABS['bert'])
  bad = [c for c in d['cases'] if tok.words(c[0]) != c[1]]
  assert not bad, bad[:5]


def test_oracle_truncation_and_threads(golden):
  g = golden('tok_bert.npz')
  tok = OracleTokenizer(VOCABS['bert'])
  a, na = tok.run(g['data'], g['sent_off'], 7, nthreads=1)
  b, nb = tok.run(g['data'], g['sent_off'], 7, nthreads=3)
  assert np.array_equal(na, np.minimum(g['ntok'], 7)) and np.array_equal(na, nb)
  for x, y in zip(compact(a, na, g['sent_off']), compact(b, nb, g['sent_off'])):
    assert np.array_equal(x, y)
