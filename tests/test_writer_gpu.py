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


@pytest.mark.parametrize('spans', [False, True])
@pytest.mark.parametrize('k', [0, 6, 12, 18, 24, 27, 30, 33])
@pytest.mark.parametrize('binned', [False, True])
def test_bert_parquet_golden(packer, tmp_path, k, binned, spans):
  from lddl_amd import writer
  case = BERT['cases'][k]
  c = case['cfg']
  if case['error']:
    pytest.skip('reference raises for this case')
  masking = c['masking']
  sh, ids, ntok = shards_from_docs(case['docs'])
  bin_size = case['bin_size'] if binned else None
  res = packer.pack(sh, ids, ntok, target_seq_length=c['max_seq'], short_seq_prob=c['ssp'],
                    duplicate_factor=c['dup'], seed=case['seed'], bin_size=bin_size, masking=masking, spans=spans)
  assert res.spans == spans
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


@pytest.mark.parametrize('spans', [False, True])
@pytest.mark.parametrize('k', range(12))
def test_codebert_parquet_golden(cpacker, tmp_path, k, spans):
  from lddl_amd import writer
  case = CODE['cases'][k]
  c = case['cfg']
  if case['error']:
    pytest.skip('reference raises for this case')
  sh, ids, ntok = shards_from_docs(case['docs'], case['ndoc'])
  res = cpacker.pack(sh, ids, ntok, target_seq_length=c['max_seq'], short_seq_prob=c['ssp'],
                     duplicate_factor=c['dup'], seed=case['seed'], codebert=True, spans=spans)
  assert res.spans == spans
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


@pytest.mark.parametrize('spans,side', [(False, False), (True, False), (True, True)])
def test_end_to_end_parquet_vs_oracle(gpu, tmp_path, spans, side):
  """synthetic corpus, several partitions (some empty), binned seq 128:
  every file's rows equal the oracle's rendering of its pairs (side: the
  writer renders and copies on a stream that is not the current one)"""
  import torch
  from lddl_amd import synth, pipeline, writer
  from oracle.oracle import OracleTokenizer
  c = synth.make_wiki(400_000, seed=77)
  pdo = pipeline.partition_by_bytes(c, 5)
  pdo = np.concatenate([[0], pdo[:3], pdo[2:]])  # an empty partition (1 -> 2 ... duplicate cut)
  pk = pipeline.Packer(pipeline.VOCAB_BERT, 0)
  sh = pipeline.upload(c, pdo, gpu)
  res = pk.run(sh, target_seq_length=128, bin_size=32, seed=99, spans=spans)
  st = None
  if side:
    st = torch.cuda.Stream(device=gpu)
    st.wait_stream(torch.cuda.current_stream())
  files = writer.write_shards(pk, res, str(tmp_path), bin_size=32, batch_rows=500, stream=st)
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
  from lddl_amd import readers
  idx, order, pdo = preprocess.plan_input(args)
  n_part = len(pdo) - 1
  in_files = preprocess.find_files_under(str(src))
  assert n_part == readers.count_partitions(in_files, readers.estimate_block_size([str(tmp_path / 'wiki')], 4))
  assert sorted(os.path.basename(f) for f in files) == sorted(
      'part.%d.parquet_%d' % (p, b) for p in range(n_part) for b in range(4))
  # the records in the plan's sampled / shuffled order are Python text-mode
  # lines (read_text's), independently of the byte-level record index
  all_recs = list(readers.iter_lines(in_files[0])) + list(readers.iter_lines(in_files[1]))
  recs = [all_recs[i] for i in preprocess.sample_order(len(all_recs), 5, 0.9)]
  assert recs == idx.texts(order)
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
  assert "'split_workers': 2" in r.stdout and ("'chunks': %d" % n_part) in r.stdout, r.stdout
  # one chunk of every partition, split as pieces on the two workers at once
  sink4 = tmp_path / 'out4'
  r4 = subprocess.run([sys.executable, '-m', 'lddl_amd.preprocess', '--sink', str(sink4), '--split-workers', '2'] +
                      common[:-1] + ['100'], cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                      capture_output=True, text=True, timeout=300)
  assert r4.returncode == 0, r4.stderr[-2000:]
  assert "'split_workers': 2" in r4.stdout and "'chunks': 1," in r4.stdout, r4.stdout
  files3, t3 = preprocess.main(preprocess.attach_args().parse_args(['--sink', str(sink3), '--split-workers', '0'] +
                                                                     common))
  assert t3['chunks'] > 1 and t['chunks'] == 1
  for f in files:
    assert _read(f) == _read(str(sink2 / os.path.basename(f))) == _read(str(sink3 / os.path.basename(f))) == \
        _read(str(sink4 / os.path.basename(f)))
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
  # (these counts are ones the reference's balancer finishes; its non-terminating
  # case is a CPU test of balance.plan: tests/test_balance.py)
  written, ns = balance.main(bargs)
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
  # two files: read_code gives one partition per file whatever --num-blocks says
  (tmp_path / 'code' / 'a.txt').write_bytes('\r\n'.join(lines[:170]).encode('utf-8'))
  (tmp_path / 'code' / 'b.txt').write_bytes('\r\n'.join(lines[170:]).encode('utf-8'))
  sink = tmp_path / 'out'
  args = preprocess.attach_args(codebert=True).parse_args(
      ['--code', str(tmp_path / 'code'), '--sink', str(sink), '--target-seq-length', '128', '--num-blocks', '2',
       '--seed', '8', '--sample-ratio', '1.0', '--split-workers', '0', '--chunk-mb', '0.1'])
  files, t = preprocess.main(args, codebert=True)
  assert sorted(os.path.basename(f) for f in files) == ['part.0.parquet', 'part.1.parquet']
  idx, order, pdo = preprocess.plan_input(args, codebert=True)
  all_recs = list(preprocess.read_records([str(tmp_path / 'code' / n) for n in ('a.txt', 'b.txt')], '\r\n'))
  recs = [all_recs[i] for i in preprocess.sample_order(len(all_recs), 8, 1.0)]
  assert recs == idx.texts(order) and len(pdo) == 3
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


def _read_dir(d):
  out = {}
  for n in sorted(os.listdir(d)):
    if n.startswith('shard-'):
      out[n] = _read(os.path.join(d, n))
  return out


def test_cli_num_shards_all_gather_over_ranks(gpu, tmp_path):
  """--num-shards: the balanced shards come straight from the packer's counts
  (one all-gather over the ranks, load_balance.py:222-233 replaced).  Two
  ranks (gloo on one GPU) write the same shard files and .num_samples.json
  as one rank, and as the standalone balancer over the same part files."""
  import json
  import socket
  import subprocess
  import sys
  from lddl_amd import synth, balance
  c = synth.make_wiki(250_000, seed=77)
  docs = c.documents()
  src = tmp_path / 'wiki' / 'en'
  src.mkdir(parents=True)
  for k in range(3):
    with open(str(src / ('wiki_%d.txt' % k)), 'w', encoding='utf-8') as f:
      for d in range(k, len(docs), 3):
        f.write('wiki-%d %s\n' % (d, ' '.join(docs[d])))
  common = ['--wikipedia', str(tmp_path / 'wiki'), '--target-seq-length', '128', '--bin-size', '64',
            '--num-blocks', '6', '--sentence-splitter', 'rules', '--seed', '3', '--split-workers', '0',
            '--num-shards', '4', '--keep-orig']
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  one, two = tmp_path / 'one', tmp_path / 'two'
  r = subprocess.run([sys.executable, '-m', 'lddl_amd.preprocess', '--sink', str(one)] + common, cwd=root,
                     capture_output=True, text=True, timeout=300)
  assert r.returncode == 0, r.stderr[-3000:]
  with socket.socket() as s:
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
  procs = []
  for rank in range(2):
    env = dict(os.environ, RANK=str(rank), WORLD_SIZE='2', LOCAL_RANK='0', MASTER_ADDR='127.0.0.1',
               MASTER_PORT=str(port), LDDL_DIST_BACKEND='gloo')
    procs.append(subprocess.Popen([sys.executable, '-m', 'lddl_amd.preprocess', '--sink', str(two)] + common,
                                  cwd=root, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
  for p in procs:
    out, err = p.communicate(timeout=300)
    assert p.returncode == 0, err[-3000:]
  a, b = _read_dir(str(one)), _read_dir(str(two))
  assert a and sorted(a) == sorted(b)
  for n in a:
    assert a[n] == b[n], n
  ns1 = json.load(open(str(one / '.num_samples.json')))
  assert ns1 == json.load(open(str(two / '.num_samples.json')))
  # the standalone balancer (counts from the parquet footers) plans the same shards
  import shutil
  parts, bal = tmp_path / 'parts', tmp_path / 'bal'
  parts.mkdir()
  for n in os.listdir(str(one)):
    if n.startswith('part.'):
      shutil.copy(str(one / n), str(parts / n))
  written, ns = balance.main(balance.attach_args().parse_args(
      ['--indir', str(parts), '--outdir', str(bal), '--num-shards', '4', '--keep-orig']), rank=0, world=1)
  assert ns == ns1
  c3 = _read_dir(str(bal))
  for n in a:
    assert c3[n] == a[n], n


def _txt_lines(path):
  with open(path, encoding='utf-8', newline='') as f:
    s = f.read()
  return s.split('\n') if s else []


@pytest.mark.parametrize('k', [0, 12, 24, 30])
@pytest.mark.parametrize('binned', [False, True])
def test_bert_txt_same_pairs_as_parquet(packer, tmp_path, k, binned):
  """--output-format txt (pretrain.py:501-531): the same rows as the parquet
  sink, in the reference's line format; {p}.txt / {p}_{b}.txt names
  (to_textfiles, binning.py:439-476), every file created, '\\n'-joined"""
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
  pq_files = writer.write_shards(packer, res, str(tmp_path / 'pq'), bin_size=bin_size, masking=masking, part_base=3)
  txt_files = writer.write_txt(packer, res, str(tmp_path / 'txt'), bin_size=bin_size, masking=masking, part_base=3,
                               batch_rows=61)
  nb = case['nbins'] if binned else 1
  assert [os.path.basename(f) for f in txt_files] == (['3_%d.txt' % b for b in range(nb)] if binned else ['3.txt'])
  for pf, tf in zip(pq_files, txt_files):
    rows = _read(pf)
    want = []
    for i in range(len(rows['A'])):
      if masking:
        pos = np.load(__import__('io').BytesIO(rows['masked_lm_positions'][i]))
        want.append('is_random_next: {} - [CLS] {} [SEP] {} [SEP] - masked_lm_positions: {} - masked_lm_labels: {} - {}'
                    .format(rows['is_random_next'][i], rows['A'][i], rows['B'][i], pos, rows['masked_lm_labels'][i],
                            rows['num_tokens'][i]))
      else:
        want.append('is_random_next: {} - [CLS] {} [SEP] {} [SEP] - {}'.format(
            rows['is_random_next'][i], rows['A'][i], rows['B'][i], rows['num_tokens'][i]))
    # (a masked_lm_positions array wider than numpy's 75-column line holds
    # newlines, as the reference's str(np.ndarray) does: compare whole files)
    with open(tf, encoding='utf-8', newline='') as f:
      assert f.read() == '\n'.join(want)
    if binned:  # binning.py:465-467: the bin is parsed back from each row's last field (num_tokens)
      for w in want:
        assert po.bin_of(int(w.split()[-1]), case['bin_size'], nb) == int(os.path.basename(tf)[:-4].split('_')[1])


def test_cli_codebert_txt(gpu, tmp_path):
  """--output-format txt for CodeBERT (pretrain_codebert.py:540-559): the
  parquet run's rows as '{id} [CLS] {doc} [SEP] {code} [SEP] - {n}'"""
  from lddl_amd import synth, preprocess
  lines = synth.make_code_lines(120, seed=4)
  (tmp_path / 'code').mkdir()
  (tmp_path / 'code' / 'a.txt').write_bytes('\r\n'.join(lines).encode('utf-8'))
  common = ['--code', str(tmp_path / 'code'), '--target-seq-length', '128', '--seed', '8', '--sample-ratio', '1.0',
            '--split-workers', '0']
  preprocess.main(preprocess.attach_args(codebert=True).parse_args(common + ['--sink', str(tmp_path / 'pq')]),
                  codebert=True)
  files, _ = preprocess.main(preprocess.attach_args(codebert=True).parse_args(
      common + ['--sink', str(tmp_path / 'txt'), '--output-format', 'txt']), codebert=True)
  assert [os.path.basename(f) for f in files] == ['0.txt']
  rows = _read(str(tmp_path / 'pq' / 'part.0.parquet'))
  want = ['{} [CLS] {} [SEP] {} [SEP] - {}'.format(i, d, c, n) for i, d, c, n in
          zip(rows['id'], rows['doc'], rows['code'], rows['num_tokens'])]
  assert want and _txt_lines(files[0]) == want


def test_cli_resume_skips_completed_chunks(gpu, tmp_path):
  """--resume: a rerun skips every chunk with a marker of the same run and
  redoes a chunk whose file went missing, with the same bytes; a rerun with
  other flags trusts no marker"""
  from lddl_amd import synth, preprocess
  c = synth.make_wiki(200_000, seed=9)
  docs = c.documents()
  src = tmp_path / 'wiki' / 'en'
  src.mkdir(parents=True)
  for k in range(3):
    with open(str(src / ('wiki_%d.txt' % k)), 'w', encoding='utf-8') as f:
      for d in range(k, len(docs), 3):
        f.write('wiki-%d %s\n' % (d, ' '.join(docs[d])))
  sink = tmp_path / 'out'
  common = ['--wikipedia', str(tmp_path / 'wiki'), '--sink', str(sink), '--target-seq-length', '128',
            '--bin-size', '64', '--sentence-splitter', 'rules', '--seed', '3', '--chunk-mb', '0.02',
            '--split-workers', '0', '--resume']
  files, t = preprocess.main(preprocess.attach_args().parse_args(common))
  assert t['chunks'] == 3 and t['chunks_skipped'] == 0
  blobs = {f: open(f, 'rb').read() for f in files}
  files2, t2 = preprocess.main(preprocess.attach_args().parse_args(common))
  assert t2['chunks_skipped'] == 3 and t2['pairs'] == t['pairs'] and sorted(files2) == sorted(files)
  gone = sorted(files)[0]
  os.remove(gone)
  files3, t3 = preprocess.main(preprocess.attach_args().parse_args(common))
  assert t3['chunks_skipped'] == 2 and sorted(files3) == sorted(files)
  assert all(open(f, 'rb').read() == blobs[f] for f in files)
  # a run without --resume and other flags rewrites the part files: the old
  # markers must not vouch for them afterwards
  plain = [a for a in common if a != '--resume'] + ['--duplicate-factor', '3']
  preprocess.main(preprocess.attach_args().parse_args(plain))
  files5, t5 = preprocess.main(preprocess.attach_args().parse_args(common))
  assert t5['chunks_skipped'] == 0 and sorted(files5) == sorted(files)
  assert all(open(f, 'rb').read() == blobs[f] for f in files)
  _, t4 = preprocess.main(preprocess.attach_args().parse_args(common + ['--duplicate-factor', '2']))
  assert t4['chunks_skipped'] == 0


def test_render_npy_matches_host(packer):
  """lddl_render_npy (the masked_lm_positions column on the GPU) against
  the host restatement npy_positions (numpy's own np.save header per
  length): rows with 0..300 positions, a row range inside the rows"""
  import ctypes
  import torch
  from types import SimpleNamespace
  from lddl_amd import _lib, writer
  rng = np.random.default_rng(3)
  k = rng.integers(0, 301, size=5000)
  k[::97] = 0
  off = np.zeros(len(k) + 1, np.int64)
  np.cumsum(k, out=off[1:])
  pos = rng.integers(0, 65536, size=int(off[-1])).astype(np.uint16)
  res = SimpleNamespace(mlm_off=torch.from_numpy(off).cuda(), mlm_pos=torch.from_numpy(pos.view(np.int16)).cuda())
  for r0, n in ((0, len(k)), (123, 2000), (len(k), 0)):
    got = writer.render_npy(packer, res, r0, n)
    exp = writer.npy_positions(off[r0:r0 + n + 1] - off[r0], pos[off[r0]:off[r0 + n]])
    assert np.array_equal(got[0], exp[0]) and np.array_equal(got[1], exp[1]), (r0, n)
  # a row longer than the header table is refused
  hdr, hlen, _ = writer.npy_header_table(packer.device)
  o = torch.empty(2, dtype=torch.int64, device='cuda')
  nb = ctypes.c_int64()
  big = int(np.argmax(k))
  rc = _lib.lib().lddl_render_npy(packer.tok.handle, ctypes.c_void_p(res.mlm_off.data_ptr()),
                                  ctypes.c_void_p(res.mlm_pos.data_ptr()), big, 1, ctypes.c_void_p(hdr.data_ptr()),
                                  hlen, int(k[big]) - 1, ctypes.c_void_p(o.data_ptr()), None, 0, ctypes.byref(nb), None)
  assert rc == -1
