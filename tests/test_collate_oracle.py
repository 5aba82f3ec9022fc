"""CPU: the collate oracle (oracle/collate_oracle.py) against the reference's
own _to_encoded_inputs outputs (tests/golden/collate_bert.json.gz,
tools/gen_golden_collate.py)."""
import gzip
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from lddl_amd import _lib
from oracle.collate_oracle import CollateOracle

VOCABS = {'bert': _lib.VOCAB_BERT, 'codebert': _lib.VOCAB_CODEBERT}


def load_cases():
  with gzip.open(os.path.join(GOLDEN, 'collate_bert.json.gz'), 'rt', encoding='utf-8') as f:
    return json.load(f)


def case_batch(c):
  if c['static']:
    return [(a, b, rn, bytes.fromhex(p), l) for a, b, rn, p, l in
            zip(c['A'], c['B'], c['is_random_next'], c['positions_npy'], c['labels_str'])]
  return list(zip(c['A'], c['B'], c['is_random_next']))


CASES = load_cases()


@pytest.mark.parametrize('k', range(len(CASES)))
def test_oracle_matches_reference(k):
  c = CASES[k]
  o = CollateOracle(VOCABS[c['vocab']])
  out = o.encode(case_batch(c), c['align'], c['ignore_index'])
  keys = ['input_ids', 'token_type_ids', 'attention_mask', 'next_sentence_labels',
          'labels' if c['static'] else 'special_tokens_mask']
  for key in keys:
    assert np.array_equal(out[key], np.asarray(c[key], np.int64)), key


def test_golden_covers_edge_cases():
  assert any(c['static'] for c in CASES) and any(not c['static'] for c in CASES)
  assert any(c['align'] == 1 for c in CASES) and any(c['ignore_index'] == -100 for c in CASES)
  unk = [np.sum(np.asarray(c['input_ids']) == 100) for c in CASES if c['vocab'] == 'bert']
  assert sum(unk) > 0  # out-of-vocab tokens exercised
  assert any('　' in a or '\xa0' in a for c in CASES for a in c['A'] + c['B'])
