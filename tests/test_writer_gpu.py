"""Parquet shards (lddl_render_strings + writer) vs the reference's rows.

Expected strings are the reference's own: ' '.join of the vocab tokens of
the golden rows (pretrain.py:348-360, pretrain_codebert.py:425-432), the
np.save bytes the reference serialised (masked_lm_positions_npy), and the
file naming / schema of pretrain.py:444-498 and binning.py:353-431.
"""
import os

import numpy as np
import pyarrow.parquet as pq
import pytest

from oracle import pack_oracle as po
from test_pack_gpu import BERT, CODE, shards_from_docs, packer, cpacker  # noqa: F401 (fixtures)

pytestmark = pytest.mark.gpu


def _vocab(path):
  with open(path, encoding='utf-8') as f:
    return [l.rstrip('\n').rstrip('\r') for l in f]


def _join(vocab, ids):
  return ' '.join(vocab[i] for i in ids)


def _read(path):
  return pq.read_table(path).to_pydict()


@pytest.mark.parametrize('k', [0, 6, 12, 18, 24, 27, 30, 33])
@pytest.mark.parametrize('binned', [False, True])
def test_bert_parquet_golden(packer, tmp_path, k, binned):
  from lddl_amd import writer
  case = BERT['cases'][k]
  c = case['cfg']
  if case['error']:
    pytest.skip('reference raises for this case')
  masking = c['masking']
  sh, ids, ntok = shards_from_docs(case['docs'])
  bin_size = case['bin_size'] if binned else None
  res = packer.pack(sh, ids, ntok, target_seq_length=c['max_seq'], short_seq_prob=c['ssp'],
                    duplicate_factor=c['dup'], seed=case['seed'], bin_size=bin_size, masking=masking)
  files = writer.write_shards(packer, res, str(tmp_path), bin_size=bin_size, masking=masking, part_base=7,
                              batch_rows=97)  # small batches: files split across render batches
  vocab = _vocab(packer.tok.vocab_file)
  exp = case['rows']
  if binned:
    order, counts = po.binned_order([r['num_tokens'] for r in exp], case['bin_size'], case['nbins'])
    exp = [exp[i] for i in order]
    names = ['part.7.parquet_%d' % b for b in range(case['nbins'])]
  else:
    counts = [len(exp)]
    names = ['part.7.parquet']
  assert [os.path.basename(f) for f in files] == names
  got = {}
  for f, n in zip(files, counts):
    t = pq.read_table(f)
    assert t.schema == writer.schema(False, masking, binned)
    assert t.num_rows == n
    for kk, v in t.to_pydict().items():
      got.setdefault(kk, []).extend(v)
  assert got['A'] == [_join(vocab, e['A']) for e in exp]
  assert got['B'] == [_join(vocab, e['B']) for e in exp]
  assert got['is_random_next'] == [e['is_random_next'] for e in exp]
  assert got['num_tokens'] == [e['num_tokens'] for e in exp]
  if binned:
    assert got['bin_id'] == [po.bin_of(e['num_tokens'], case['bin_size'], case['nbins']) for e in exp]
  if masking:
    assert got['masked_lm_positions'] == [bytes.fromhex(e['masked_lm_positions_npy']) for e in exp]
    assert got['masked_lm_labels'] == [_join(vocab, e['masked_lm_labels']) for e in exp]


@pytest.mark.parametrize('k', range(12))
def test_codebert_parquet_golden(cpacker, tmp_path, k):
  from lddl_amd import writer
  case = CODE['cases'][k]
  c = case['cfg']
  if case['error']:
    pytest.skip('reference raises for this case')
  sh, ids, ntok = shards_from_docs(case['docs'], case['ndoc'])
  res = cpacker.pack(sh, ids, ntok, target_seq_length=c['max_seq'], short_seq_prob=c['ssp'],
                     duplicate_factor=c['dup'], seed=case['seed'], codebert=True)
  doc_ids = ['py_%d' % d for d in range(len(case['docs']))]
  files = writer.write_shards(cpacker, res, str(tmp_path), codebert=True, doc_ids=doc_ids)
  assert [os.path.basename(f) for f in files] == ['part.0.parquet']
  t = pq.read_table(files[0])
  assert t.schema == writer.schema(True, False, False)
  vocab = _vocab(cpacker.tok.vocab_file)
  got = t.to_pydict()
  exp = case['rows']
  assert got['id'] == [e['id'] for e in exp]
  assert got['doc'] == [_join(vocab, e['doc']) for e in exp]
  assert got['code'] == [_join(vocab, e['code']) for e in exp]
  assert got['num_tokens'] == [e['num_tokens'] for e in exp]


def test_end_to_end_parquet_vs_oracle(gpu, tmp_path):
  """synthetic corpus, several partitions (some empty), binned seq 128:
  every file's rows equal the oracle's rendering of its pairs"""
  from lddl_amd import synth, pipeline, writer
  from oracle.oracle import OracleTokenizer
  c = synth.make_wiki(400_000, seed=77)
  pdo = pipeline.partition_by_bytes(c, 5)
  pdo = np.concatenate([[0], pdo[:3], pdo[2:]])  # an empty partition (1 -> 2 ... duplicate cut)
  pk = pipeline.Packer(pipeline.VOCAB_BERT, 0)
  sh = pipeline.upload(c, pdo, gpu)
  res = pk.run(sh, target_seq_length=128, bin_size=32, seed=99)
  files = writer.write_shards(pk, res, str(tmp_path), bin_size=32, batch_rows=500)
  assert len(files) == (len(pdo) - 1) * 4
  oids, ontok = OracleTokenizer(pipeline.VOCAB_BERT).run(c.data, c.sent_off, 512, nthreads=8)
  exp = po.run_bert_shards(c, oids, ontok, pdo, 128, 0.1, 5, 99, 32)
  vocab = _vocab(pipeline.VOCAB_BERT)
  for p, rows in enumerate(exp):
    for b in range(4):
      got = _read(os.path.join(str(tmp_path), 'part.%d.parquet_%d' % (p, b)))
      want = [r for r in rows if po.bin_of(r[3], 32, 4) == b]
      assert got['A'] == [_join(vocab, r[0]) for r in want]
      assert got['B'] == [_join(vocab, r[1]) for r in want]
      assert got['is_random_next'] == [bool(r[2]) for r in want]
      assert got['num_tokens'] == [r[3] for r in want]
