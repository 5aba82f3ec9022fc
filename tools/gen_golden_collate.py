#!/usr/bin/env python3
"""Golden vectors for the training-time collate, produced by the REFERENCE's
own ``_to_encoded_inputs`` (lddl/torch/bert.py:69-153) with a
transformers.BertTokenizerFast over the local vocab files (run HERE only;
/root/reference is read, never copied).

Batches: rows of vocab tokens (incl. '##' pieces, specials, out-of-vocab
strings -> [UNK]), separated by runs of ASCII and Unicode whitespace (str.split
semantics), empty segments, ragged lengths; alignment 8 / 1 / 64, ignore_index
-1 / -100; static-masking batches carry np.save positions (the reference's
serialize_np_array) and label strings.  Dynamic batches record the reference's
special_tokens_mask (the input of _mask_tokens).

Writes tests/golden/collate_bert.json.gz (data only).
"""
import gzip
import json
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, '/root/reference')
import transformers  # noqa: E402
import lddl.torch.bert as ref  # noqa: E402
from lddl.utils import serialize_np_array  # noqa: E402

from lddl_amd import _lib  # noqa: E402

SEPS = [' ', ' ', ' ', '  ', '\t', '\n', '　', '\xa0', ' ', '\x1f', ' ', ' \r\n ']
OOV = ['zzqxj', 'ünïcödé', 'héllo', '日本語', '\U0001F600', 'a​b', 'foo##', '##', '[sep]', 'Hello']


def vocab(path):
  with open(path, encoding='utf-8') as f:
    return [l.rstrip('\n') for l in f]


def seg(rng, V, n, fancy):
  toks = []
  for _ in range(n):
    r = rng.random()
    if fancy and r < 0.08:
      toks.append(rng.choice(OOV))
    elif fancy and r < 0.10:
      toks.append(rng.choice(['[UNK]', '[MASK]', '[SEP]', '[CLS]', '[PAD]']))
    else:
      toks.append(V[rng.randrange(len(V))])
  if not fancy:
    return ' '.join(toks)
  s = ''
  for i, t in enumerate(toks):
    s += (rng.choice(SEPS) if i else (rng.choice(['', '', ' ', '\t']))) + t
  return s + rng.choice(['', '', ' ', '\n'])


def batch(rng, V, n, max_len, fancy, static):
  out = []
  for _ in range(n):
    na = rng.randrange(0, max_len)
    nb = rng.randrange(0, max(1, max_len - na))
    a, b = seg(rng, V, na, fancy), seg(rng, V, nb, fancy)
    rn = rng.random() < 0.5
    if not static:
      out.append((a, b, rn))
      continue
    ta, tb = a.split(), b.split()
    n_tok = len(ta) + len(tb) + 3
    cand = [i for i in range(n_tok) if i != 0 and i != len(ta) + 1 and i != n_tok - 1]
    k = min(len(cand), max(1, int(round(n_tok * 0.15))))
    pos = sorted(rng.sample(cand, k)) if cand else []
    toks = ['[CLS]'] + ta + ['[SEP]'] + tb + ['[SEP]']
    labels = ' '.join(toks[p] if rng.random() < 0.9 else rng.choice(V) for p in pos)
    out.append((a, b, rn, serialize_np_array(np.asarray(pos, dtype=np.uint16)), labels))
  return out


def main():
  rng = random.Random(20261016)
  cases = []
  for vf, tag in ((_lib.VOCAB_BERT, 'bert'), (_lib.VOCAB_CODEBERT, 'codebert')):
    V = vocab(vf)
    tok = transformers.BertTokenizerFast(vf)
    specs = [(16, 60, True, False, 8, -1), (16, 60, True, True, 8, -1), (8, 200, False, False, 8, -1),
             (8, 200, False, True, 1, -100), (4, 509, False, False, 64, -1), (1, 3, True, False, 8, -1),
             (12, 30, True, True, 1, -1)]
    if tag == 'codebert':
      specs = specs[:3]
    for n, ml, fancy, static, align, ign in specs:
      b = batch(rng, V, n, ml, fancy, static)
      enc = ref._to_encoded_inputs(b, tok, sequence_length_alignment=align, ignore_index=ign)
      case = {'vocab': tag, 'align': align, 'ignore_index': ign, 'static': static,
              'A': [s[0] for s in b], 'B': [s[1] for s in b], 'is_random_next': [bool(s[2]) for s in b]}
      if static:
        case['positions_npy'] = [s[3].hex() for s in b]
        case['labels_str'] = [s[4] for s in b]
      for k, v in enc.items():
        case[k] = v.tolist()
      cases.append(case)
  path = os.path.join(ROOT, 'tests', 'golden', 'collate_bert.json.gz')
  with gzip.open(path, 'wt', encoding='utf-8') as f:
    json.dump(cases, f)
  print('wrote %s: %d batches' % (path, len(cases)))


if __name__ == '__main__':
  main()
