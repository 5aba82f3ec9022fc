#!/usr/bin/env python3
"""Golden vectors for the tokenizer (run HERE only; needs HF tokenizers).

Oracle: ``transformers.BertTokenizerFast(vocab_file)`` exactly as the reference
builds it (``lddl/dask/bert/pretrain.py:584-587``), called the way the
reference calls it (``pretrain.py:79-80``: ``tokenize(s, max_length=512,
truncation=True)``).  transformers 5.x ignores those kwargs, so the 4.16.2
per-sentence truncation is applied here as ``[:512]``.

Writes tests/golden/tok_<vocab>.npz with the raw sentence bytes, offsets, the
expected ids (compact CSR) and per-sentence counts.
"""
import os
import sys

import numpy as np
import transformers

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lddl_amd import synth  # noqa: E402

VOCABS = {
    'bert': os.path.join(ROOT, 'lddl_amd', 'data', 'bert_vocab.txt'),
    'codebert': os.path.join(ROOT, 'lddl_amd', 'data', 'codebert_52000_vocab.txt'),
}

EDGE = [
    '', ' ', 'a', 'A', 'Hello, World!', 'foo[SEP]bar', '[sep]', '[SEP]', '[SEP][SEP]', '[MASK]x',
    '[CLS', '[CLS]]', '[[PAD]]', '[UNK]', 'x[UNK]y', 'a☃b', 'naïve café', 'İstanbul', 'ΣΑΣ',
    '中文 字', '中文字abc中', '한국어', '서울시', '😀', '🚀ok', 'a\u0007b', 'a\x00b', '�',
    'x​y', 'a b', 'a　b', 'a b', 'a\u0085b', 'tab\there', 'nl\nhere',
    'cr\rhere', '﻿bom', 'ﬁne', 'Ⅻ', 'ｆｕｌｌ', 'ß', 'ǅemal', '𝐛𝐨𝐥𝐝', 'm̀́̂', 'e' + '́' * 150,
    'x' * 100, 'x' * 101, 'y' * 300, 'ab' * 60, '##', '#hash', '###', 'a##b', '...', '!!?',
    "don't", 'e.g.', 'U.S.A.', '3.14159', '1,000,000', '$5', '100%', '<b>bold</b>',
    'unaffable', 'undesirableness', 'electroencephalographically', 'pneumonoultramicroscopic',
    'Ωmega', 'Ǆ', 'ǆ', 'ᾼ', 'ﬀ', 'Ⓐ', '㎏', '𝔘𝔫𝔦', '\U0001D15E\U0001D16D\U0001D165',
    '\U0001D16D́\U0001D165', 'abु́cd', 'ꙮ', 'ё', 'Ё', 'İi̇', 'ǰ',
    ' '.join(['word'] * 600), ' '.join(['unaffable'] * 200),
    'def f(x):', 'return x**2 + 1', 'self.assertEqual(a, b)', 'import numpy as np',
    '    indented    ', 'snake_case_name', 'camelCaseName', 'CONSTANT_VALUE', '0xDEADBEEF',
]


def fuzz(rng, n):
  import json
  d = json.load(open(os.path.join(ROOT, 'tests', 'golden', 'normalize_fuzz.json')))
  cases = [c[0] for c in d['cases']]
  out = []
  for _ in range(n):
    k = int(rng.integers(1, 5))
    out.append(' '.join(cases[int(rng.integers(0, len(cases)))] for _ in range(k)))
  return out


def main():
  rng = np.random.default_rng(7)
  wiki = synth.make_wiki(1_200_000, seed=11)
  wiki_s = [wiki.sentence(i) for i in range(wiki.n_sent)][:8000]
  code = synth.make_code(600, seed=12)
  code_s = [code.sentence(i) for i in range(code.n_sent)][:8000]
  for name, path in VOCABS.items():
    tok = transformers.BertTokenizerFast(path)
    bt = tok.backend_tokenizer
    sents = EDGE + fuzz(rng, 2000) + (wiki_s if name == 'bert' else code_s) + \
        (code_s[:1500] if name == 'bert' else wiki_s[:1500])
    enc = bt.encode_batch(sents, add_special_tokens=False)
    ids = [e.ids[:512] for e in enc]
    # cross-check the reference calling pattern on a sample
    for s, i in zip(sents[:400], ids[:400]):
      assert tok.convert_tokens_to_ids(tok.tokenize(s, max_length=512, truncation=True))[:512] == i
    c = synth.corpus_from_sentences(sents, [0, len(sents)])
    cnt = np.array([len(i) for i in ids], dtype=np.int32)
    flat = np.array([x for i in ids for x in i], dtype=np.int32)
    out = os.path.join(ROOT, 'tests', 'golden', 'tok_%s.npz' % name)
    np.savez_compressed(out, data=c.data, sent_off=c.sent_off, ids=flat, ntok=cnt,
                        tokenizers=np.array(__import__('tokenizers').__version__))
    nb = c.nbytes
    print(name, len(sents), 'sentences', nb, 'bytes', flat.size, 'tokens',
          '%.2f B/token' % (nb / max(1, flat.size)), os.path.getsize(out), 'file bytes')


if __name__ == '__main__':
  main()
