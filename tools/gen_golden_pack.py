#!/usr/bin/env python3
"""Golden vectors for pair packing + binning, produced by the REFERENCE's own
functions (run HERE only; /root/reference is read, never copied).

lddl.dask.bert.pretrain / pretrain_codebert import once dask / nltk are
stubbed; we then call their create_pairs_from_document
directly and restate the 5-line _to_partition_pairs closure
(pretrain.py:386-402) with an explicit random.seed per partition.  Masking
uses vocab_words in vocab-file order (the reference's tuple(vocab.keys()) is
hash-ordered).  Binning restates binning.py:72-75.

Writes tests/golden/pack_bert.json.gz, pack_codebert.json.gz (data only).
"""
import gzip
import json
import os
import random
import sys
import unittest.mock as mock

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

for m in ['dask', 'dask.bag', 'dask.distributed', 'dask.highlevelgraph', 'dask.base', 'dask.bag.core',
          'dask.delayed', 'dask.utils', 'dask.dataframe', 'dask.dataframe.core', 'dask.dataframe.io',
          'dask.dataframe.io.parquet', 'dask.dataframe.io.parquet.core', 'dask.dataframe.io.parquet.arrow',
          'dask.bytes', 'tlz', 'nltk', 'nltk.tokenize', 'dask_mpi']:
  sys.modules[m] = mock.MagicMock()
sys.path.insert(0, '/root/reference')
import lddl.dask.bert.pretrain as ref  # noqa: E402
import lddl.dask.bert.pretrain_codebert as refc  # noqa: E402
from lddl.utils import deserialize_np_array  # noqa: E402

from lddl_amd import synth  # noqa: E402
from oracle.oracle import OracleTokenizer  # noqa: E402


def vocab(path):
  with open(path, encoding='utf-8') as f:
    return [l.rstrip('\n') for l in f]


def tokenized_docs(corpus, vf):
  ot = OracleTokenizer(vf)
  ids, ntok = ot.run(corpus.data, corpus.sent_off, 512, nthreads=8)
  base = corpus.sent_off[0]
  docs = []
  for d in range(corpus.n_doc):
    sents = []
    for s in range(corpus.doc_sent_off[d], corpus.doc_sent_off[d + 1]):
      o = int(corpus.sent_off[s] - base)
      sents.append([int(x) for x in ids[o:o + ntok[s]]])
    docs.append(sents)
  return docs


def ref_bert_partition(docs_ids, V, seed, max_seq, ssp, dup, masking, ratio):
  documents = []
  for k, d in enumerate(docs_ids):
    sents = tuple(ref.Sentence(tuple(V[t] for t in s)) for s in d if len(s) > 0)
    if sents:
      documents.append(ref.Document('doc%d' % k, sents))
  documents = tuple(documents)
  random.seed(seed)
  pairs = []
  for _ in range(dup):
    for di in range(len(documents)):
      pairs.extend(ref.create_pairs_from_document(documents, di, max_seq_length=max_seq, short_seq_prob=ssp,
                                                  masking=masking, masked_lm_ratio=ratio,
                                                  vocab_words=tuple(V)))
  random.shuffle(pairs)
  return pairs


def main():
  Vb = vocab(os.path.join(ROOT, 'lddl_amd', 'data', 'bert_vocab.txt'))
  idx = {t: i for i, t in enumerate(Vb)}
  wiki = synth.make_wiki(400_000, seed=21)
  docs = tokenized_docs(wiki, os.path.join(ROOT, 'lddl_amd', 'data', 'bert_vocab.txt'))
  rng = np.random.default_rng(5)
  cases = []
  # partitions: consecutive docs; plus edge partitions
  parts = [docs[0:30], docs[30:45], docs[45:46], [[d[0]] for d in docs[46:60]],
           [[[1037] * 600], [[1037] * 3, [1996] * 2]],  # long sentence + tiny doc
           [[[2003]], [[2003]], [[2003]]]]  # 1-token sentences
  for cfg in [dict(max_seq=128, ssp=0.1, dup=5, masking=False), dict(max_seq=512, ssp=0.1, dup=2, masking=False),
              dict(max_seq=128, ssp=0.5, dup=2, masking=False), dict(max_seq=16, ssp=0.1, dup=2, masking=False),
              dict(max_seq=128, ssp=0.1, dup=2, masking=True), dict(max_seq=512, ssp=0.1, dup=1, masking=True)]:
    for pi, part in enumerate(parts):
      seed = 12345 + pi
      try:
        pairs = ref_bert_partition(part, Vb, seed, cfg['max_seq'], cfg['ssp'], cfg['dup'], cfg['masking'], 0.15)
        err = None
      except AssertionError:
        pairs, err = [], 'AssertionError'
      rows = []
      for p in pairs:
        row = {'A': [idx[t] for t in p['A'].split(' ')] if p['A'] else [],
               'B': [idx[t] for t in p['B'].split(' ')] if p['B'] else [],
               'is_random_next': bool(p['is_random_next']), 'num_tokens': int(p['num_tokens'])}
        if cfg['masking']:
          row['masked_lm_positions'] = [int(x) for x in deserialize_np_array(p['masked_lm_positions'])]
          row['masked_lm_positions_npy'] = p['masked_lm_positions'].hex()
          row['masked_lm_labels'] = [idx[t] for t in p['masked_lm_labels'].split(' ')]
        rows.append(row)
      # binning (binning.py:72-75) for bin_size = max_seq // 4
      bs = cfg['max_seq'] // 4
      nb = cfg['max_seq'] // bs
      bins = [min((r['num_tokens'] - 1) // bs, nb - 1) for r in rows]
      cases.append({'cfg': cfg, 'seed': seed, 'docs': part, 'rows': rows, 'error': err,
                    'bin_size': bs, 'nbins': nb, 'bins': bins})
  with gzip.open(os.path.join(ROOT, 'tests', 'golden', 'pack_bert.json.gz'), 'wt') as f:
    json.dump({'generator': 'tools/gen_golden_pack.py', 'reference': 'lddl/dask/bert/pretrain.py:241-402',
               'seed_rule': 'random.seed(seed) before each partition', 'cases': cases}, f)
  print('bert cases', len(cases), sum(len(c['rows']) for c in cases), 'rows')

  # ---------------- CodeBERT ----------------
  Vc = vocab(os.path.join(ROOT, 'lddl_amd', 'data', 'codebert_52000_vocab.txt'))
  cidx = {t: i for i, t in enumerate(Vc)}
  code = synth.make_code(120, seed=22)
  cdocs = tokenized_docs(code, os.path.join(ROOT, 'lddl_amd', 'data', 'codebert_52000_vocab.txt'))
  ndoc = [int(x) for x in code.doc_nseg_doc]
  ccases = []
  cparts = [(cdocs[0:40], ndoc[0:40]), (cdocs[40:80], ndoc[40:80]),
            ([[[5] * 200] + s[ndoc[80]:] for s in cdocs[80:84]], [1] * 4),  # long first docstring line
            ([[[7] * 3, [8] * 2, [9] * 70, [10] * 3] + [[11] * 5] * 2], [3])]
  for cfg in [dict(max_seq=512, ssp=0.1, dup=1), dict(max_seq=128, ssp=0.1, dup=2), dict(max_seq=128, ssp=0.9, dup=1)]:
    for pi, (part, nd) in enumerate(cparts):
      seed = 777 + pi
      cps = []
      for k, (d, n) in enumerate(zip(part, nd)):
        ds = tuple(refc.Sentence(tuple(Vc[t] for t in s)) for s in d[:n] if len(s) > 0)
        cs = tuple(refc.Sentence(tuple(Vc[t] for t in s)) for s in d[n:] if len(s) > 0)
        cp = refc.CodePair('py_%d' % k, refc.Document(cs), refc.Document(ds))
        if len(cp) > 0:
          cps.append(cp)
      cps = tuple(cps)
      random.seed(seed)
      rows, err = [], None
      try:
        pairs = []
        for _ in range(cfg['dup']):
          for di in range(len(cps)):
            pairs.extend(refc.create_pairs_from_document(cps, di, max_seq_length=cfg['max_seq'],
                                                         short_seq_prob=cfg['ssp']))
        random.shuffle(pairs)
        for p in pairs:
          rows.append({'id': p['id'], 'doc': [cidx[t] for t in p['doc'].split(' ')] if p['doc'] else [],
                       'code': [cidx[t] for t in p['code'].split(' ')] if p['code'] else [],
                       'num_tokens': int(p['num_tokens'])})
      except IndexError:
        err = 'IndexError'
      ccases.append({'cfg': cfg, 'seed': seed, 'docs': part, 'ndoc': nd, 'rows': rows, 'error': err})
  with gzip.open(os.path.join(ROOT, 'tests', 'golden', 'pack_codebert.json.gz'), 'wt') as f:
    json.dump({'generator': 'tools/gen_golden_pack.py',
               'reference': 'lddl/dask/bert/pretrain_codebert.py:343-477', 'cases': ccases}, f)
  print('codebert cases', len(ccases), sum(len(c['rows']) for c in ccases), 'rows',
        [c['error'] for c in ccases])


if __name__ == '__main__':
  main()
