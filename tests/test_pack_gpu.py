"""HIP packer (BERT NSP / CodeBERT / binning / materialise) vs golden rows
from the reference functions and vs the oracle restatement."""
import numpy as np
import pytest
import torch

from oracle import pack_oracle as po
from oracle.oracle import OracleTokenizer
from test_pack_oracle import BERT, CODE

pytestmark = pytest.mark.gpu


def shards_from_docs(docs, nseg=None, part_doc_off=None, device='cuda'):
  """pre-tokenised docs (lists of id lists) -> ShardSet + ids/ntok tensors"""
  from lddl_amd.pipeline import ShardSet
  sents = [s for d in docs for s in d]
  ntok = np.array([len(s) for s in sents], dtype=np.int32)
  off = np.zeros(len(sents) + 1, dtype=np.int64)
  np.cumsum(ntok, out=off[1:])
  ids = np.array([t for s in sents for t in s] + [0] * 16, dtype=np.uint16)  # (+16: materialize's 16-B loads)
  dso = np.zeros(len(docs) + 1, dtype=np.int64)
  np.cumsum([len(d) for d in docs], out=dso[1:])
  pdo = np.array(part_doc_off if part_doc_off is not None else [0, len(docs)], dtype=np.int64)
  sh = ShardSet(torch.zeros(int(off[-1]) + 16, dtype=torch.uint8, device=device),
                torch.from_numpy(off).to(device), torch.from_numpy(dso).to(device),
                torch.from_numpy(pdo).to(device),
                None if nseg is None else torch.tensor(nseg, dtype=torch.int32, device=device), int(off[-1]))
  return sh, torch.from_numpy(ids.view(np.int16)).to(device), torch.from_numpy(ntok).to(device)


@pytest.fixture(scope='module')
def packer(gpu):
  from lddl_amd.pipeline import Packer, VOCAB_BERT
  return Packer(VOCAB_BERT, 0)


@pytest.fixture(scope='module')
def cpacker(gpu):
  from lddl_amd.pipeline import Packer, VOCAB_CODEBERT
  return Packer(VOCAB_CODEBERT, 0)


@pytest.mark.parametrize('k', [i for i, c in enumerate(BERT['cases']) if not c['cfg']['masking']])
@pytest.mark.parametrize('binned', [False, True])
def test_bert_golden(packer, k, binned):
  case = BERT['cases'][k]
  c = case['cfg']
  sh, ids, ntok = shards_from_docs(case['docs'])
  kw = dict(target_seq_length=c['max_seq'], short_seq_prob=c['ssp'], duplicate_factor=c['dup'],
            seed=case['seed'], bin_size=case['bin_size'] if binned else None)
  if case['error']:
    with pytest.raises(AssertionError):
      packer.pack(sh, ids, ntok, **kw)
    return
  res = packer.pack(sh, ids, ntok, **kw)
  rows = res.rows()
  exp = case['rows']
  if binned:
    order, counts = po.binned_order([r['num_tokens'] for r in exp], case['bin_size'], case['nbins'])
    exp = [exp[i] for i in order]
    assert res.bin_count.cpu().numpy().tolist() == [counts]
  assert len(rows) == len(exp)
  for (p, a, b, fl, bn, tok), e in zip(rows, exp):
    assert (a, b, bool(fl & 1), len(tok)) == (e['A'], e['B'], e['is_random_next'], e['num_tokens'])
    assert tok[0] == packer.tok.cls_id and tok[1 + len(a)] == packer.tok.sep_id and tok[-1] == packer.tok.sep_id
    if binned:
      assert bn == po.bin_of(e['num_tokens'], case['bin_size'], case['nbins'])


@pytest.mark.parametrize('k', range(len(CODE['cases'])))
def test_codebert_golden(cpacker, k):
  case = CODE['cases'][k]
  c = case['cfg']
  sh, ids, ntok = shards_from_docs(case['docs'], case['ndoc'])
  kw = dict(target_seq_length=c['max_seq'], short_seq_prob=c['ssp'], duplicate_factor=c['dup'],
            seed=case['seed'], codebert=True)
  if case['error']:
    with pytest.raises(IndexError):
      cpacker.pack(sh, ids, ntok, **kw)
    return
  res = cpacker.pack(sh, ids, ntok, **kw)
  rows = res.rows()
  assert len(rows) == len(case['rows'])
  for (p, a, b, fl, bn, tok), e in zip(rows, case['rows']):
    assert (a, b, len(tok)) == (e['doc'], e['code'], e['num_tokens'])


@pytest.mark.parametrize('caps,mat', [(None, None), ('8192,512,8192', None), ('0,0,256', None), (None, '1'),
                                      (None, 'spans')])
@pytest.mark.parametrize('seq,bin_size,nparts', [(128, 32, 7), (512, 64, 3), (128, None, 1)])
def test_bert_end_to_end_vs_oracle(gpu, monkeypatch, seq, bin_size, nparts, caps, mat):
  """caps: the wave packer's per-partition arrays in global memory (default),
  all in LDS, and order/num_tokens in LDS with a capacity some partitions
  exceed (mixed paths in one launch).  mat: the chunked materialize and
  compaction kernels (default), the per-partition / per-sentence ones (1),
  or no materialisation: the rows as spans of the dense ids (lddl_row_spans)."""
  from lddl_amd import synth, pipeline
  if caps:
    monkeypatch.setenv('LDDL_PACK_CAPS', caps)
  if mat == '1':
    monkeypatch.setenv('LDDL_MAT_ALGO', mat)
  c = synth.make_wiki(600_000, seed=seq + nparts)
  res = pipeline.run_bert(c, target_seq_length=seq, bin_size=bin_size, n_partitions=nparts, seed=999,
                          check_host=True, spans=mat == 'spans')
  assert res.spans == (mat == 'spans')
  oids, ontok = OracleTokenizer(pipeline.VOCAB_BERT).run(c.data, c.sent_off, 512, nthreads=8)
  assert np.array_equal(res.ntok_host, ontok)
  exp = po.run_bert_shards(c, oids, ontok, res.part_doc_off, seq, 0.1, 5, 999, bin_size)
  pipeline.assert_same_pairs(res, exp)
  # bin counts agree with the rows
  nb = res.nbins
  bc = res.bin_count.cpu().numpy()
  for p, part in enumerate(exp):
    cnt = np.bincount([po.bin_of(r[3], bin_size or (1 << 30), nb) for r in part], minlength=nb)
    assert np.array_equal(bc[p], cnt)


@pytest.mark.parametrize('seed', [0, 2**32 - 2, 2**40 + 3])
def test_bert_partition_seeds_vs_oracle(gpu, seed):
  """random.seed(seed + p) for seeds of one and two 32-bit key words
  (init_by_array's klen 1 / 2; 2**32 - 2 + p crosses the boundary) and 0"""
  from lddl_amd import synth, pipeline
  c = synth.make_wiki(300_000, seed=17)
  res = pipeline.run_bert(c, target_seq_length=128, bin_size=32, n_partitions=4, seed=seed, check_host=True)
  oids, ontok = OracleTokenizer(pipeline.VOCAB_BERT).run(c.data, c.sent_off, 512, nthreads=8)
  exp = po.run_bert_shards(c, oids, ontok, res.part_doc_off, 128, 0.1, 5, seed, 32)
  pipeline.assert_same_pairs(res, exp)


@pytest.mark.parametrize('nparts', [2, 5])
def test_wikibooks_seq512_bin64_vs_oracle(gpu, nparts):
  """BASELINE config C5 at a size the oracle finishes quickly: a Wikipedia +
  Books-style corpus (--wikipedia + --books, readers.py:73-99; books are long
  documents of short sentences with dialogue and contractions), seq 512,
  --bin-size 64, duplicate factor 5."""
  from lddl_amd import synth, pipeline
  c = synth.make_wikibooks(1_500_000, seed=40 + nparts)
  res = pipeline.run_bert(c, target_seq_length=512, bin_size=64, n_partitions=nparts, seed=2024, check_host=True)
  oids, ontok = OracleTokenizer(pipeline.VOCAB_BERT).run(c.data, c.sent_off, 512, nthreads=8)
  assert np.array_equal(res.ntok_host, ontok)
  exp = po.run_bert_shards(c, oids, ontok, res.part_doc_off, 512, 0.1, 5, 2024, 64)
  pipeline.assert_same_pairs(res, exp)
  bc = res.bin_count.cpu().numpy()
  for p, part in enumerate(exp):
    assert np.array_equal(bc[p], np.bincount([po.bin_of(r[3], 64, 8) for r in part], minlength=8))


@pytest.mark.parametrize('mat', [None, '1', 'spans'])
def test_codebert_end_to_end_vs_oracle(gpu, monkeypatch, mat):
  from lddl_amd import synth, pipeline
  if mat == '1':
    monkeypatch.setenv('LDDL_MAT_ALGO', mat)
  c = synth.make_code(400, seed=31)
  pdo = pipeline.partition_by_bytes(c, 3)
  res = pipeline.run_bert(c, vocab_file=pipeline.VOCAB_CODEBERT, target_seq_length=512, bin_size=64,
                          part_doc_off=pdo, seed=42, duplicate_factor=1, codebert=True, check_host=True,
                          spans=mat == 'spans')
  assert res.spans == (mat == 'spans')
  oids, ontok = OracleTokenizer(pipeline.VOCAB_CODEBERT).run(c.data, c.sent_off, 512, nthreads=8)
  assert np.array_equal(res.ntok_host, ontok)
  rows = res.rows()
  g = 0
  for p in range(len(pdo) - 1):
    docs, nd = [], []
    for d in range(pdo[p], pdo[p + 1]):
      ss = [list(map(int, oids[c.sent_off[s]:c.sent_off[s] + ontok[s]]))
            for s in range(c.doc_sent_off[d], c.doc_sent_off[d + 1])]
      k = int(c.doc_nseg_doc[d])
      ds = [s for s in ss[:k] if s]
      cs = [s for s in ss[k:] if s]
      if cs:
        docs.append(ds + cs)
        nd.append(len(ds))
    pairs = po.partition_pairs(docs, 42 + p, lambda D, di, r: po.codebert_pairs(D, nd, di, 512, 0.1, r), 1)
    exp = []
    for (doc_s, code_s, dw, cw) in pairs:
      dt = [t for (d, s) in doc_s for t in docs[d][s]][dw[0]:dw[1]]
      ct = [t for (d, s) in code_s for t in docs[d][s]][cw[0]:cw[1]]
      exp.append((dt, ct, len(dt) + len(ct) + (3 if nd[code_s[0][0]] else 2)))
    order, _ = po.binned_order([e[2] for e in exp], 64, 8)
    for i in order:
      pp, a, b, fl, bn, tok = rows[g]
      assert (pp, a, b, len(tok)) == (p, exp[i][0], exp[i][1], exp[i][2])
      g += 1
  assert g == len(rows)


@pytest.mark.parametrize('spans', [False, True])
def test_many_partitions_and_empty_partitions(packer, spans):
  # partitions with zero docs and docs with empty sentences; as span rows,
  # partitions of fewer than 64 rows share a row-spans wave
  docs = [[[5, 6, 7], [], [8, 9]], [[]], [[10] * 40, [11] * 30, [12] * 50], [[13] * 3]] * 20
  pdo = [0, 0, 5, 5, 17, 40, 80, 80]
  sh, ids, ntok = shards_from_docs(docs, part_doc_off=pdo)
  res = packer.pack(sh, ids, ntok, target_seq_length=64, duplicate_factor=2, seed=7, bin_size=16, spans=spans)
  assert res.spans == spans
  rows = res.rows()
  fdocs = [[s for s in d if s] for d in docs]
  exp = []
  for p in range(len(pdo) - 1):
    D = [d for d in fdocs[pdo[p]:pdo[p + 1]] if d]
    prs = po.partition_pairs(D, 7 + p, lambda X, di, r: po.bert_pairs(X, di, 64, 0.1, r), 2)
    rr = [po.pair_tokens(D, pr) for pr in prs]
    order, _ = po.binned_order([len(a) + len(b) + 3 for a, b, _ in rr], 16, 4)
    exp += [(p,) + rr[i] for i in order]
  assert [(r[0], r[1], r[2], bool(r[3] & 1)) for r in rows] == [(p, a, b, rn) for p, a, b, rn in exp]


# ---------------------------------------------------------------- masking --
MASK = (0.15, 30522, 101, 102, 103)  # ratio, |vocab|, [CLS], [SEP], [MASK] of bert-base-uncased


@pytest.mark.parametrize('spans', [False, True])
@pytest.mark.parametrize('k', [i for i, c in enumerate(BERT['cases']) if c['cfg']['masking']])
@pytest.mark.parametrize('binned', [False, True])
def test_bert_masked_golden(packer, k, binned, spans):
  """--masking rows against the reference's create_masked_lm_predictions
  (rows materialised and masked in place, or spans + lddl_masked_lm_spans)."""
  case = BERT['cases'][k]
  c = case['cfg']
  sh, ids, ntok = shards_from_docs(case['docs'])
  kw = dict(target_seq_length=c['max_seq'], short_seq_prob=c['ssp'], duplicate_factor=c['dup'],
            seed=case['seed'], bin_size=case['bin_size'] if binned else None, masking=True, spans=spans)
  if case['error']:
    with pytest.raises(AssertionError):
      packer.pack(sh, ids, ntok, **kw)
    return
  res = packer.pack(sh, ids, ntok, **kw)
  rows = res.rows()
  exp = case['rows']
  if binned:
    order, _ = po.binned_order([r['num_tokens'] for r in exp], case['bin_size'], case['nbins'])
    exp = [exp[i] for i in order]
  assert len(rows) == len(exp)
  assert res.n_masked == sum(len(e['masked_lm_positions']) for e in exp)
  for (p, a, b, fl, bn, tok, pos, lab), e in zip(rows, exp):
    assert (a, b, bool(fl & 1), len(tok)) == (e['A'], e['B'], e['is_random_next'], e['num_tokens'])
    assert pos == e['masked_lm_positions'] and lab == e['masked_lm_labels']
    # serialize_np_array(np.asarray(positions, np.uint16)) bytes
    assert np.asarray(pos, dtype=np.uint16).tobytes().hex() in e['masked_lm_positions_npy']


# (seq 1024: the MASK = 2 packer instantiation, MaskLds<1024>, 10-bit shuffle draws)
@pytest.mark.parametrize('spans', [False, True])
@pytest.mark.parametrize('seq,bin_size,nparts', [(128, 32, 5), (512, 64, 2), (1024, 128, 2)])
def test_bert_masked_end_to_end_vs_oracle(gpu, seq, bin_size, nparts, spans):
  from lddl_amd import synth, pipeline
  c = synth.make_wiki(500_000, seed=seq + 3 * nparts)
  res = pipeline.run_bert(c, target_seq_length=seq, bin_size=bin_size, n_partitions=nparts, seed=4242,
                          check_host=True, masking=True, spans=spans)
  assert res.spans == spans
  oids, ontok = OracleTokenizer(pipeline.VOCAB_BERT).run(c.data, c.sent_off, 512, nthreads=8)
  assert np.array_equal(res.ntok_host, ontok)
  exp = po.run_bert_shards(c, oids, ontok, res.part_doc_off, seq, 0.1, 5, 4242, bin_size, masking=MASK)
  pipeline.assert_same_pairs(res, exp)
  # statistical sanity of the 80/10/10 split over the whole run
  rows = res.rows()
  n = sum(len(r[6]) for r in rows)
  n_mask = sum(1 for r in rows for q in r[6] if r[5][q] == 103)
  assert 0.75 < n_mask / n < 0.85


# seq 512 at a high masking ratio: 0.5 puts up to 256 picks per pair in the
# MASK = 1 lists (their capacity, MLM_PICKS_1), 0.6 up to 307 picks, which
# the launch sends to the MASK = 2 instantiation
@pytest.mark.parametrize('ratio', [0.5, 0.6])
def test_bert_masked_high_ratio_vs_oracle(gpu, ratio):
  from lddl_amd import synth, pipeline
  c = synth.make_wiki(300_000, seed=77)
  res = pipeline.run_bert(c, target_seq_length=512, bin_size=64, n_partitions=2, seed=99, check_host=True,
                          masking=True, masked_lm_ratio=ratio, spans=True)
  oids, ontok = OracleTokenizer(pipeline.VOCAB_BERT).run(c.data, c.sent_off, 512, nthreads=8)
  exp = po.run_bert_shards(c, oids, ontok, res.part_doc_off, 512, 0.1, 5, 99, 64, masking=(ratio,) + MASK[1:])
  pipeline.assert_same_pairs(res, exp)
  assert max(len(r[6]) for r in res.rows()) > 200


def test_bert_masked_special_tokens_and_arena_regrow(gpu, monkeypatch):
  """Sentences holding literal [CLS]/[SEP] tokens take the explicit candidate
  list (pretrain.py:187-190); a tiny initial arena forces the regrow path."""
  from lddl_amd.pipeline import Packer, VOCAB_BERT
  monkeypatch.setenv('LDDL_MLM_CAP', '1000')
  pk = Packer(VOCAB_BERT, 0)
  rng = np.random.default_rng(3)
  docs = []
  for d in range(60):
    doc = []
    for s in range(int(rng.integers(1, 9))):
      n = int(rng.integers(1, 40))
      sent = [int(x) for x in rng.integers(999, 30000, n)]
      for _ in range(int(rng.integers(0, 3))):
        sent[int(rng.integers(0, n))] = int(rng.choice([101, 102, 103]))
      doc.append(sent)
    docs.append(doc)
  pdo = [0, 20, 41, 60]
  sh, ids, ntok = shards_from_docs(docs, part_doc_off=pdo)
  res = pk.pack(sh, ids, ntok, target_seq_length=64, duplicate_factor=3, seed=11, bin_size=16, masking=True)
  exp = []
  for p in range(len(pdo) - 1):
    D = docs[pdo[p]:pdo[p + 1]]
    prs = po.partition_pairs(D, 11 + p, lambda X, di, r: po.bert_pairs(X, di, 64, 0.1, r, MASK), 3)
    rr = []
    for pr in prs:
      a, b, rn = po.pair_tokens(D, pr)
      ma, mb, pos, lab = pr[5]
      rr.append((ma, mb, rn, len(a) + len(b) + 3, pos, lab))
    order, _ = po.binned_order([r[3] for r in rr], 16, 4)
    exp.append([rr[i] for i in order])
  from lddl_amd.pipeline import assert_same_pairs
  assert_same_pairs(res, exp)


def codebert_oracle_rows(docs, ndoc, pdo, seq, ssp, dup, seed, bin_size, nbins):
  """oracle/pack_oracle.py over pre-tokenised CodeBERT documents: the rows
  (partition, doc tokens, code tokens, num_tokens) in output order and the
  per-(partition, bin) counts; raises IndexError like the reference's
  _truncate_seq quirk (pretrain_codebert.py:236-247)"""
  rows, counts = [], []
  for p in range(len(pdo) - 1):
    D, nd = [], []
    for d in range(pdo[p], pdo[p + 1]):  # empty segments / docs without code dropped (:143-161)
      ds = [x for x in docs[d][:ndoc[d]] if x]
      cs = [x for x in docs[d][ndoc[d]:] if x]
      if cs:
        D.append(ds + cs)
        nd.append(len(ds))
    pairs = po.partition_pairs(D, seed + p, lambda X, di, r: po.codebert_pairs(X, nd, di, seq, ssp, r), dup)
    exp = []
    for (doc_s, code_s, dw, cw) in pairs:
      dt = [t for (d, s) in doc_s for t in D[d][s]][dw[0]:dw[1]]
      ct = [t for (d, s) in code_s for t in D[d][s]][cw[0]:cw[1]]
      exp.append((dt, ct, len(dt) + len(ct) + (3 if nd[code_s[0][0]] else 2)))
    order, cnt = po.binned_order([e[2] for e in exp], bin_size, nbins)
    rows += [(p,) + exp[i] for i in order]
    counts.append(cnt)
  return rows, counts


@pytest.mark.parametrize('seq,ssp,dup', [(512, 0.1, 1), (128, 0.0, 2), (512, 1.0, 1), (128, 0.3, 3)])
def test_codebert_long_documents_vs_oracle(cpacker, seq, ssp, dup):
  """Documents with > 64 code and docstring segments (multi-window scans),
  long segments (truncation rounds across MT twists), empty segments: the
  wave packer against the oracle (oracle/pack_oracle.py codebert_pairs,
  itself pinned by the reference goldens)."""
  rng = np.random.default_rng(seq + dup)
  docs, ndoc = [], []
  for d in range(60):
    nds = int(rng.choice([0, 1, 3, 70]))
    ncs = int(rng.choice([1, 2, 40, 130]))
    segs = []
    for q in range(nds + ncs):
      n = int(rng.choice([0, 1, 5, 12, 40, 90])) if q < nds else int(rng.choice([0, 2, 9, 30, 200]))
      segs.append([int(x) for x in rng.integers(1000, 2000, n)])
    if not any(segs[nds:]):
      segs[-1] = [1500] * 7
    docs.append(segs)
    ndoc.append(nds)
  pdo = [0, 13, 13, 40, 60]
  sh, ids, ntok = shards_from_docs(docs, ndoc, part_doc_off=pdo)
  try:
    exp, counts = codebert_oracle_rows(docs, ndoc, pdo, seq, ssp, dup, 77, seq // 4, 4)
  except IndexError:
    with pytest.raises(IndexError):
      cpacker.pack(sh, ids, ntok, target_seq_length=seq, short_seq_prob=ssp, duplicate_factor=dup, seed=77,
                   codebert=True, bin_size=seq // 4)
    return
  res = cpacker.pack(sh, ids, ntok, target_seq_length=seq, short_seq_prob=ssp, duplicate_factor=dup, seed=77,
                     codebert=True, bin_size=seq // 4)
  rows = res.rows()
  assert len(rows) == len(exp)
  for (p, a, b, fl, bn, tok), e in zip(rows, exp):
    assert (p, a, b, len(tok)) == e
  assert res.bin_count.cpu().numpy().tolist() == counts


def test_masked_special_flags_from_tokenizer(gpu):
  """With masking, sentences holding a literal [CLS] / [SEP] token build an
  explicit candidate list (pretrain.py:187-190).  The tokenizer writes those
  per-sentence flags (scan kernel + serial fallback) and a masked pack over
  the same id buffers reuses them; a pack over a copy of the ids recomputes
  them with a pass over the ids: both must give identical rows."""
  from lddl_amd import pipeline
  from lddl_amd.synth import corpus_from_sentences
  rng = np.random.default_rng(5)
  words = ['the', 'cat', 'sat', 'on', 'mat', 'running', 'unbelievable', '[CLS]', '[SEP]', '[MASK]', 'x[SEP]y',
           'é', 'naïve', '中文']
  sents, dso = [], [0]
  for d in range(300):
    for s in range(int(rng.integers(1, 12))):
      sents.append(' '.join(rng.choice(words, int(rng.integers(1, 40)))))
    dso.append(len(sents))
  c = corpus_from_sentences(sents, dso)
  pk = pipeline.Packer(pipeline.VOCAB_BERT, 0, masking=True)
  sh = pipeline.upload(c, pipeline.partition_by_bytes(c, 3), torch.device('cuda', 0))
  ids, ntok, toff = pk.tokenize(sh)
  kw = dict(target_seq_length=128, duplicate_factor=2, seed=3, bin_size=32, masking=True)
  a = pk.pack(sh, ids, ntok, toff, **kw).rows()
  b = pk.pack(sh, ids.clone(), ntok, toff, **kw).rows()
  assert len(a) == len(b) and a == b


@pytest.mark.parametrize('codebert,nbytes', [(False, 500_000), (True, 0), (False, 6_000_000)])
def test_row_spans_equal_materialized_rows(gpu, codebert, nbytes):
  """lddl_row_spans describes exactly lddl_materialize's rows: the same
  row offsets, lengths, flags, bins, partitions and bin counts, and the
  tokens the spans select from the dense ids equal the materialised rows
  (6 MB: > 64 row-span blocks, so their XCD-aware order is in play)"""
  from lddl_amd import synth, pipeline
  c = synth.make_code(300, seed=8) if codebert else synth.make_wiki(nbytes, seed=8)
  vocab = pipeline.VOCAB_CODEBERT if codebert else pipeline.VOCAB_BERT
  pdo = pipeline.partition_by_bytes(c, 4 if nbytes <= 500_000 else 23)
  pk = pipeline.Packer(vocab, 0)
  sh = pipeline.upload(c, pdo, gpu)
  ids, ntok, toff = pk.tokenize(sh)
  kw = dict(target_seq_length=256, bin_size=32, seed=5, codebert=codebert, duplicate_factor=1 if codebert else 3)
  m = pk.pack(sh, ids, ntok, toff, **kw)
  mt = m.host_tokens()
  mcopy = {k: getattr(m, k)[:m.n_pairs + (1 if k == 'tok_off' else 0)].cpu().numpy().copy()
           for k in ('tok_off', 'len0', 'len1', 'flags', 'bins', 'part')}
  mbc = m.bin_count.cpu().numpy().copy()
  s = pk.pack(sh, ids, ntok, toff, spans=True, **kw)
  assert s.spans and s.tokens is None and s.n_pairs == m.n_pairs and s.n_pairs > 0
  if nbytes > 500_000:
    assert (s.n_pairs + 255) // 256 >= 64 and ((s.n_pairs + 255) // 256) % 8, s.n_pairs  # (rounded-up grid)
  for k, v in mcopy.items():
    assert np.array_equal(getattr(s, k)[:s.n_pairs + (1 if k == 'tok_off' else 0)].cpu().numpy(), v), k
  assert np.array_equal(s.bin_count.cpu().numpy(), mbc)
  assert np.array_equal(s.host_tokens(), mt)


@pytest.mark.parametrize('codebert', [False, True])
def test_upload_pieces_equals_upload_of_concat(gpu, codebert):
  """a chunk's pieces staged straight into the pinned H2D buffers equal the
  upload of their host concatenation"""
  import torch
  from lddl_amd import synth, pipeline, preprocess, writer
  if codebert:
    recs = synth.make_code_lines(31, seed=4)
    split = None
  else:
    recs = ['wiki-%d %s' % (i, ' '.join(d)) for i, d in enumerate(synth.make_wiki(1 << 15, seed=6).documents())]
    split = preprocess.sentence_splitter('rules')[0]
  cuts = [0, 2, 2, len(recs) // 2, len(recs)]
  parts = [preprocess.split_records(recs[a:b], codebert, split) for a, b in zip(cuts[:-1], cuts[1:])]
  ids = [writer.str_array(p[1]) for p in parts] if codebert else [p[1] for p in parts]
  whole, _ = preprocess.concat_corpora([p[0] for p in parts], ids)
  pdo = np.array([0, 1, whole.n_doc // 2, whole.n_doc], np.int64)
  dev = torch.device('cuda', 0)
  a = pipeline.upload(whole, pdo, dev)
  b = pipeline.upload_pieces([p[0] for p in parts], pdo, dev)
  torch.cuda.synchronize()
  assert a.nbytes == b.nbytes
  for f in ('data', 'sent_off', 'doc_sent_off', 'part_doc_off'):
    assert torch.equal(getattr(a, f), getattr(b, f)), f
  assert (a.doc_nseg_doc is None) == (b.doc_nseg_doc is None)
  if codebert:
    assert torch.equal(a.doc_nseg_doc, b.doc_nseg_doc)
