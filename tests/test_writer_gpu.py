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


def _bin_rows(rows, bin_size, nbins):
  return [[r for r in rows if po.bin_of(r[-1], bin_size, nbins) == b] for b in range(nbins)]


def test_cli_bert_end_to_end(gpu, tmp_path):
  """preprocess_bert_pretrain drop-in: text files -> part.{i}.parquet_{b},
  rows equal to the oracle pipeline on the same sampled / shuffled /
  sentence-split corpus; then the load balancer over the written files"""
  from lddl_amd import synth, preprocess, pipeline, balance
  from oracle.oracle import OracleTokenizer
  c = synth.make_wiki(300_000, seed=123)
  docs = c.documents()
  src = tmp_path / 'wiki' / 'en'
  src.mkdir(parents=True)
  for k in range(2):
    with open(str(src / ('wiki_%d.txt' % k)), 'w', encoding='utf-8') as f:
      for d in range(k, len(docs), 2):
        f.write('wiki-%d %s\n' % (d, ' '.join(docs[d])))
  sink = tmp_path / 'out'
  args = preprocess.attach_args().parse_args(
      ['--wikipedia', str(tmp_path / 'wiki'), '--sink', str(sink), '--target-seq-length', '128', '--bin-size', '32',
       '--num-blocks', '4', '--sentence-splitter', 'rules', '--seed', '5', '--split-workers', '0'])
  files, t = preprocess.main(args)
  assert sorted(os.path.basename(f) for f in files) == sorted(
      'part.%d.parquet_%d' % (p, b) for p in range(4) for b in range(4))
  # several pipeline chunks split ahead by forked worker processes give the
  # same files: the CLI in a fresh process (its workers fork before the GPU
  # is touched, as in production), and inline chunks in this one
  import subprocess
  import sys
  sink2, sink3 = tmp_path / 'out2', tmp_path / 'out3'
  common = ['--wikipedia', str(tmp_path / 'wiki'), '--target-seq-length', '128', '--bin-size', '32',
            '--num-blocks', '4', '--sentence-splitter', 'rules', '--seed', '5', '--chunk-mb', '0.05']
  r = subprocess.run([sys.executable, '-m', 'lddl_amd.preprocess', '--sink', str(sink2), '--split-workers', '2'] +
                     common, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), capture_output=True,
                     text=True, timeout=300)
  assert r.returncode == 0, r.stderr[-2000:]
  assert "'split_workers': 2" in r.stdout and "'chunks': 4" in r.stdout, r.stdout
  files3, t3 = preprocess.main(preprocess.attach_args().parse_args(['--sink', str(sink3), '--split-workers', '0'] +
                                                                     common))
  assert t3['chunks'] > 1 and t['chunks'] == 1
  for f in files:
    assert _read(f) == _read(str(sink2 / os.path.basename(f))) == _read(str(sink3 / os.path.basename(f)))
  recs = preprocess.sample_shuffle(preprocess.read_records(preprocess.find_files_under(str(src))), 5, 0.9)
  pdo = preprocess.partition_records(recs, num_blocks=4)
  corpus, ids = preprocess.split_records(recs, splitter=preprocess._rule_split)
  oids, ontok = OracleTokenizer(pipeline.VOCAB_BERT).run(corpus.data, corpus.sent_off, 512, nthreads=8)
  exp = po.run_bert_shards(corpus, oids, ontok, pdo, 128, 0.1, 5, 5, 32)
  vocab = _vocab(pipeline.VOCAB_BERT)
  for p, rows in enumerate(exp):
    for b, want in enumerate(_bin_rows(rows, 32, 4)):
      got = _read(str(sink / ('part.%d.parquet_%d' % (p, b))))
      assert got['A'] == [_join(vocab, r[0]) for r in want]
      assert got['B'] == [_join(vocab, r[1]) for r in want]
      assert got['num_tokens'] == [r[3] for r in want]
  # load balancer over the written shards: every row lands exactly once
  bargs = balance.attach_args().parse_args(['--indir', str(sink), '--outdir', str(tmp_path / 'bal'),
                                            '--num-shards', '3', '--keep-orig'])
  try:
    written, ns = balance.main(bargs)
  except RuntimeError:
    pytest.skip('counts hit the reference load balancer non-termination case')
  for b in range(4):
    n_in = sum(len(_bin_rows(rows, 32, 4)[b]) for rows in exp)
    assert sum(v for k, v in ns.items() if k.endswith('_%d' % b)) == n_in
    got = sorted(a for k in range(3) for a in _read(str(tmp_path / 'bal' / ('shard-%d.parquet_%d' % (k, b))))['A'])
    assert got == sorted(_join(vocab, r[0]) for rows in exp for r in _bin_rows(rows, 32, 4)[b])


def test_cli_codebert_end_to_end(gpu, tmp_path):
  from lddl_amd import synth, preprocess, pipeline
  from oracle.oracle import OracleTokenizer
  lines = synth.make_code_lines(300, seed=9)
  (tmp_path / 'code').mkdir()
  (tmp_path / 'code' / 'a.txt').write_bytes('\r\n'.join(lines).encode('utf-8'))
  sink = tmp_path / 'out'
  args = preprocess.attach_args(codebert=True).parse_args(
      ['--code', str(tmp_path / 'code'), '--sink', str(sink), '--target-seq-length', '128', '--num-blocks', '2',
       '--seed', '8', '--sample-ratio', '1.0', '--split-workers', '0', '--chunk-mb', '0.1'])
  files, t = preprocess.main(args, codebert=True)
  assert sorted(os.path.basename(f) for f in files) == ['part.0.parquet', 'part.1.parquet']
  recs = preprocess.sample_shuffle(
      preprocess.read_records([str(tmp_path / 'code' / 'a.txt')], linedelimiter='\r\n'), 8, 1.0)
  pdo = preprocess.partition_records(recs, num_blocks=2)
  c, ids = preprocess.split_records(recs, codebert=True)
  oids, ontok = OracleTokenizer(pipeline.VOCAB_CODEBERT).run(c.data, c.sent_off, 512, nthreads=8)
  vocab = _vocab(pipeline.VOCAB_CODEBERT)
  for p in range(2):
    docs, nd, dmap = [], [], []
    for d in range(pdo[p], pdo[p + 1]):
      ss = [list(map(int, oids[c.sent_off[s]:c.sent_off[s] + ontok[s]]))
            for s in range(c.doc_sent_off[d], c.doc_sent_off[d + 1])]
      k = int(c.doc_nseg_doc[d])
      ds, cs = [s for s in ss[:k] if s], [s for s in ss[k:] if s]
      if cs:
        docs.append(ds + cs)
        nd.append(len(ds))
        dmap.append(d)
    pairs = po.partition_pairs(docs, 8 + p, lambda D, di, r: po.codebert_pairs(D, nd, di, 128, 0.1, r), 1)
    got = _read(str(sink / ('part.%d.parquet' % p)))
    want_id, want_doc, want_code = [], [], []
    for (doc_s, code_s, dw, cw) in pairs:
      want_doc.append(_join(vocab, [t for (d, s) in doc_s for t in docs[d][s]][dw[0]:dw[1]]))
      want_code.append(_join(vocab, [t for (d, s) in code_s for t in docs[d][s]][cw[0]:cw[1]]))
      want_id.append(ids[dmap[code_s[0][0]]])
    assert got['doc'] == want_doc and got['code'] == want_code and got['id'] == want_id
