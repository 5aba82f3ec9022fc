"""TEST INFRASTRUCTURE ONLY -- the CPU checker for lddl_amd.loader's GPU collate.
Never imported by lddl_amd/.

Restates lddl/torch/bert.py:69-153 `_to_encoded_inputs` with numpy (the
reference builds torch tensors row by row with a HF tokenizer):
  * tokens of a segment = Python str.split() (bert.py:82-83);
  * ids via vocab lookup, [UNK] for a miss (tokenizer.convert_tokens_to_ids,
    bert.py:106-109);
  * batch_seq_len = max(len(A)+len(B)+3) rounded up to the alignment
    (bert.py:94-101);
  * token_type_ids 1 on [len(A)+2, len(A)+len(B)+3) (bert.py:111-113),
    attention_mask 1 on [0, len(A)+len(B)+3) (bert.py:115);
  * static: labels = ignore_index, labels[positions] = ids(labels.split())
    (bert.py:117-121); else special_tokens_mask at 0, len(A)+1 and
    [len(A)+len(B)+2, ...) (bert.py:122-126).
Pinned by tests/golden/collate_bert.json.gz (the reference's own function,
tools/gen_golden_collate.py).
"""
import io

import numpy as np


class CollateOracle:

  def __init__(self, vocab_file):
    with open(vocab_file, encoding='utf-8') as f:
      toks = [l.rstrip('\n') for l in f]
    self.vocab = {}
    for i, t in enumerate(toks):
      self.vocab[t] = i  # a duplicate line: last id wins (HF WordPiece vocab map)
    self.unk = self.vocab['[UNK]']
    self.cls = self.vocab['[CLS]']
    self.sep = self.vocab['[SEP]']

  def ids(self, tokens):
    return [self.vocab.get(t, self.unk) for t in tokens]

  def encode(self, batch, sequence_length_alignment=8, ignore_index=-1):
    static = len(batch[0]) > 3
    As = [s[0].split() for s in batch]
    Bs = [s[1].split() for s in batch]
    L = max(len(a) + len(b) + 3 for a, b in zip(As, Bs))
    L = ((L - 1) // sequence_length_alignment + 1) * sequence_length_alignment
    n = len(batch)
    input_ids = np.zeros((n, L), np.int64)
    tt = np.zeros((n, L), np.int64)
    am = np.zeros((n, L), np.int64)
    lab = np.full((n, L), ignore_index, np.int64) if static else np.zeros((n, L), np.int64)
    for r, (a, b) in enumerate(zip(As, Bs)):
      toks = ['[CLS]'] + a + ['[SEP]'] + b + ['[SEP]']
      input_ids[r, :len(toks)] = self.ids(toks)
      tt[r, len(a) + 2:len(a) + len(b) + 3] = 1
      am[r, :len(a) + len(b) + 3] = 1
      if static:
        pos = np.load(io.BytesIO(batch[r][3])).astype(np.int64)
        lab[r, pos] = self.ids(batch[r][4].split())
      else:
        lab[r, 0] = 1
        lab[r, len(a) + 1] = 1
        lab[r, len(a) + len(b) + 2:] = 1
    out = {'input_ids': input_ids, 'token_type_ids': tt, 'attention_mask': am,
           'next_sentence_labels': np.asarray([bool(s[2]) for s in batch], np.int64)}
    out['labels' if static else 'special_tokens_mask'] = lab
    return out
