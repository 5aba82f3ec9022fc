"""HIP tokenizer vs the golden vectors (tokenizers 0.22.2) and vs the oracle."""
import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle.oracle import OracleTokenizer, compact
from test_oracle_golden import VOCABS

pytestmark = pytest.mark.gpu


def sparse_of_dense(ids, ntok, tok_off, sent_off, nbytes):
  """the dense CSR ids placed at their sentences' byte offsets (the oracle's
  layout, oracle.compact reads it), after checking the CSR invariants"""
  assert tok_off[0] == 0 and np.array_equal(np.diff(tok_off), ntok)
  total = int(tok_off[-1])
  sp = np.zeros(nbytes + 16, dtype=np.uint16)
  starts = np.asarray(sent_off[:-1]) - sent_off[0]
  idx = np.repeat(starts, ntok) + (np.arange(total) - np.repeat(tok_off[:-1], ntok))
  sp[idx] = ids[:total]
  return sp


def run_hip(tok, data, sent_off, max_tok=512):
  """lddl_tokenize's dense output, in the oracle's sparse layout"""
  d = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).cuda()
  o = torch.from_numpy(np.ascontiguousarray(sent_off)).cuda()
  ids, ntok, toff = tok.tokenize_device(d, o, max_tok)
  torch.cuda.synchronize()
  n = len(sent_off) - 1
  ntok = ntok.cpu().numpy()[:n]
  ids = ids.cpu().numpy().view(np.uint16)
  return sparse_of_dense(ids, ntok, toff.cpu().numpy()[:n + 1], sent_off, len(data)), ntok


@pytest.mark.parametrize('name', ['bert', 'codebert'])
@pytest.mark.parametrize('max_tok', [512, 9])
def test_hip_tokenize_matches_golden(gpu, golden, name, max_tok):
  from lddl_amd.tokenizer import Tokenizer
  g = golden('tok_%s.npz' % name)
  tok = Tokenizer(VOCABS[name])
  ids, ntok = run_hip(tok, g['data'], g['sent_off'], max_tok)
  assert np.array_equal(ntok, np.minimum(g['ntok'], max_tok))
  exp = np.split(g['ids'], np.cumsum(g['ntok'])[:-1])
  got = compact(ids, ntok, g['sent_off'])
  bad = [i for i, (a, b) in enumerate(zip(exp, got)) if not np.array_equal(a[:max_tok], b)]
  assert not bad, bad[:10]


def test_hip_tokenize_matches_oracle_synthetic(gpu):
  from lddl_amd import synth
  from lddl_amd.tokenizer import Tokenizer
  c = synth.make_wiki(8_000_000, seed=5)
  tok = Tokenizer(VOCABS['bert'])
  ids, ntok = run_hip(tok, c.data, c.sent_off)
  oids, ontok = OracleTokenizer(VOCABS['bert']).run(c.data, c.sent_off, 512, nthreads=8)
  assert np.array_equal(ntok, ontok)
  mask = np.zeros(c.nbytes, dtype=bool)
  starts = c.sent_off[:-1] - c.sent_off[0]
  # compare every emitted id position
  idx = np.repeat(starts, ntok) + (np.arange(ntok.sum()) - np.repeat(np.cumsum(ntok) - ntok, ntok))
  assert np.array_equal(ids[idx].astype(np.int64), oids[idx].astype(np.int64))
  del mask


def test_hip_tokenize_code_corpus_codebert_vocab(gpu):
  from lddl_amd import synth
  from lddl_amd.tokenizer import Tokenizer
  c = synth.make_code(3000, seed=9)
  tok = Tokenizer(VOCABS['codebert'])
  ids, ntok = run_hip(tok, c.data, c.sent_off)
  oids, ontok = OracleTokenizer(VOCABS['codebert']).run(c.data, c.sent_off, 512, nthreads=8)
  assert np.array_equal(ntok, ontok)
  for a, b in zip(compact(ids, ntok, c.sent_off), compact(oids, ontok, c.sent_off)):
    assert np.array_equal(a.astype(np.int64), b.astype(np.int64))


def test_hip_tokenize_edge_sizes(gpu):
  from lddl_amd.tokenizer import Tokenizer
  tok = Tokenizer(VOCABS['bert'])
  sents = ['', 'a', ' ', '[SEP]', 'x' * 5000, ' '.join(['hello'] * 3000), 'ab' * 400]
  got = tok.encode_batch(sents)
  ot = OracleTokenizer(VOCABS['bert'])
  from lddl_amd.synth import corpus_from_sentences
  c = corpus_from_sentences(sents, [0, len(sents)])
  oids, ontok = ot.run(c.data, c.sent_off)
  assert [list(map(int, x)) for x in compact(oids, ontok, c.sent_off)] == got
  assert tok.tokenize('Hello, World! foo[SEP]bar') == ['hello', ',', 'world', '!', 'foo', '[SEP]', 'bar']
  # a shard of 1 sentence and of 0 sentences
  assert tok.encode_batch(['x']) == [[tok.vocab['x']]]
  assert tok.encode_batch([]) == []


def adversarial_sentences(rng, n):
  """Mixtures that stress the window path: empty / 1-byte sentences, specials
  at every offset, multi-byte chars across window edges, >256-byte words,
  90-110 char words, ccc>0 survivors, CJK, controls."""
  import json
  import os
  from conftest import GOLDEN
  fz = [c[0] for c in json.load(open(os.path.join(GOLDEN, 'normalize_fuzz.json')))['cases']]
  atoms = ['a', 'the', 'Hello', ',', '.', ' ', '  ', '[SEP]', '[MASK]', '[CLS', '[sep]', 'naïve', 'İ', '中文',
           '한국어', '😀', '\x07', '\t', 'ﬁ', '\U0001D16D\U0001D165', 'm̀́', ' ', '##', 'x' * 300,
           'ab' * 55, 'q' * 99, 'q' * 101, 'é' * 120, 'unaffable', 'electroencephalographically' * 3]
  out = []
  for _ in range(n):
    r = rng.random()
    if r < 0.05:
      out.append('')
    elif r < 0.1:
      out.append(str(rng.choice(list('ab[.'))))
    else:
      k = int(rng.integers(1, 60))
      parts = []
      for _ in range(k):
        if rng.random() < 0.15:
          parts.append(fz[int(rng.integers(0, len(fz)))])
        else:
          parts.append(atoms[int(rng.integers(0, len(atoms)))])
        parts.append(' ' if rng.random() < 0.7 else '')
      out.append(''.join(parts).strip())
  return out


# '5t': tok5 with its WordPiece by trie walk (LDDL_WP_ALGO=trie, the A/B option);
# '5s': tok5 whose scan probes its two-choice whole-word table (LDDL_SCAN_TABLE=1)
ALGOS = ['0', '5', '5t', '5s', '6']


def _set_algo(monkeypatch, algo):
  monkeypatch.setenv('LDDL_TOKENIZE_ALGO', algo[0])
  if algo.endswith('t'):
    monkeypatch.setenv('LDDL_WP_ALGO', 'trie')
  else:
    monkeypatch.delenv('LDDL_WP_ALGO', raising=False)
  if algo.endswith('s'):
    monkeypatch.setenv('LDDL_SCAN_TABLE', '1')
  else:
    monkeypatch.delenv('LDDL_SCAN_TABLE', raising=False)


@pytest.mark.parametrize('algo', ALGOS)
@pytest.mark.parametrize('name', ['bert', 'codebert'])
def test_hip_tokenize_adversarial_vs_oracle(gpu, monkeypatch, algo, name):
  from lddl_amd.synth import corpus_from_sentences
  from lddl_amd.tokenizer import Tokenizer
  _set_algo(monkeypatch, algo)
  rng = np.random.default_rng(int(algo[0]) * 7 + len(name) + len(algo))
  sents = adversarial_sentences(rng, 6000)
  c = corpus_from_sentences(sents, [0, len(sents)])
  tok = Tokenizer(VOCABS[name])
  for max_tok in (512, 3):
    ids, ntok = run_hip(tok, c.data, c.sent_off, max_tok)
    oids, ontok = OracleTokenizer(VOCABS[name]).run(c.data, c.sent_off, max_tok, nthreads=8)
    bad = [i for i in range(len(sents)) if ntok[i] != ontok[i]]
    assert not bad, [(i, repr(sents[i][:80]), ntok[i], ontok[i]) for i in bad[:5]]
    for i, (a, b) in enumerate(zip(compact(ids, ntok, c.sent_off), compact(oids, ontok, c.sent_off))):
      assert np.array_equal(a.astype(np.int64), b.astype(np.int64)), (i, repr(sents[i][:80]))


@pytest.mark.parametrize('algo', ALGOS)
def test_hip_tokenize_algos_agree_on_wiki(gpu, monkeypatch, algo):
  from lddl_amd import synth
  from lddl_amd.tokenizer import Tokenizer
  _set_algo(monkeypatch, algo)
  c = synth.make_wiki(3_000_000, seed=17)
  ids, ntok = run_hip(Tokenizer(VOCABS['bert']), c.data, c.sent_off)
  oids, ontok = OracleTokenizer(VOCABS['bert']).run(c.data, c.sent_off, 512, nthreads=8)
  assert np.array_equal(ntok, ontok)
  for a, b in zip(compact(ids, ntok, c.sent_off), compact(oids, ontok, c.sent_off)):
    assert np.array_equal(a.astype(np.int64), b.astype(np.int64))


@pytest.mark.parametrize('env', [{'LDDL_SPLIT_SEG': '97'}, {'LDDL_SPLIT_CHUNKS': '3'},
                                 {'LDDL_SPLIT_SEG': '61', 'LDDL_SPLIT_CHUNKS': '40'}])
@pytest.mark.parametrize('name', ['bert', 'codebert'])
def test_hip_tokenize_split_segments_and_capacity(gpu, monkeypatch, env, name):
  """The split tokenizer (v5) over many small segments (seams between
  segments) and with too few WordPiece record chunks (tiles that run out of
  record capacity go to the exact fallback kernel): still exact."""
  from lddl_amd import synth
  from lddl_amd.tokenizer import Tokenizer
  monkeypatch.setenv('LDDL_TOKENIZE_ALGO', '5')
  for k, v in env.items():
    monkeypatch.setenv(k, v)
  c = synth.make_wiki(2_000_000, seed=29) if name == 'bert' else synth.make_code(1500, seed=31)
  for max_tok in (512, 5):
    ids, ntok = run_hip(Tokenizer(VOCABS[name]), c.data, c.sent_off, max_tok)
    oids, ontok = OracleTokenizer(VOCABS[name]).run(c.data, c.sent_off, max_tok, nthreads=8)
    assert np.array_equal(ntok, ontok)
    for a, b in zip(compact(ids, ntok, c.sent_off), compact(oids, ontok, c.sent_off)):
      assert np.array_equal(a.astype(np.int64), b.astype(np.int64))


@pytest.mark.parametrize('seg', ['1', '97'])
@pytest.mark.parametrize('name', ['bert', 'codebert'])
def test_hip_tokenize_lane_segments(gpu, monkeypatch, seg, name):
  """The lane tokenizer (v6) over many small segments: staging, offset scan
  and compaction continue across segment seams; max_tok 512 and 5."""
  from lddl_amd import synth
  from lddl_amd.tokenizer import Tokenizer
  monkeypatch.setenv('LDDL_TOKENIZE_ALGO', '6')
  monkeypatch.setenv('LDDL_SPLIT_SEG', seg)
  c = synth.make_wiki(600_000, seed=33) if name == 'bert' else synth.make_code(600, seed=35)
  for max_tok in (512, 5):
    ids, ntok = run_hip(Tokenizer(VOCABS[name]), c.data, c.sent_off, max_tok)
    oids, ontok = OracleTokenizer(VOCABS[name]).run(c.data, c.sent_off, max_tok, nthreads=8)
    assert np.array_equal(ntok, ontok)
    for a, b in zip(compact(ids, ntok, c.sent_off), compact(oids, ontok, c.sent_off)):
      assert np.array_equal(a.astype(np.int64), b.astype(np.int64))


def test_repeated_calls_reuse_scratch(gpu):
  """one Tokenizer, scratch reused across calls: a second corpus after a
  first one (record slots, piece counts and entry buffers hold the first
  call's values) and the same corpus twice give the oracle's result -- a
  word moved to a new record chunk with its sentence keeps no stale count"""
  from lddl_amd import synth
  from lddl_amd.tokenizer import Tokenizer
  tok = Tokenizer(VOCABS['bert'])
  a = synth.make_wiki(6_000_000, seed=21)
  b = synth.make_wiki(5_000_000, seed=22)
  run_hip(tok, a.data, a.sent_off)
  oids, ontok = OracleTokenizer(VOCABS['bert']).run(b.data, b.sent_off, 512, nthreads=8)
  for _ in range(2):
    ids, ntok = run_hip(tok, b.data, b.sent_off)
    assert np.array_equal(ntok, ontok)
    starts = b.sent_off[:-1] - b.sent_off[0]
    idx = np.repeat(starts, ntok) + (np.arange(ntok.sum()) - np.repeat(np.cumsum(ntok) - ntok, ntok))
    assert np.array_equal(ids[idx].astype(np.int64), oids[idx].astype(np.int64))


def test_packer_ids_buffer_grows_past_the_estimate(gpu):
  """Packer.tokenize sizes ids by Packer.ids_estimate (not the byte count);
  a corpus with more tokens than that (punctuation: one token per byte) is
  re-run into a buffer of its exact total, with the same ids as the oracle;
  a caller buffer that is too small raises CapacityError"""
  from lddl_amd.pipeline import Packer, ShardSet
  from lddl_amd.tokenizer import CapacityError
  sents = [('!' * 400) if k % 5 else 'Hello, world!! a b c.' for k in range(2500)]
  enc = [s.encode() for s in sents]
  off = np.zeros(len(enc) + 1, np.int64)
  np.cumsum([len(b) for b in enc], out=off[1:])
  data = np.frombuffer(b''.join(enc), np.uint8)
  pk = Packer(VOCABS['bert'])
  assert pk.ids_estimate(len(data)) < len(data) // 2
  d = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).cuda()
  o = torch.from_numpy(off).cuda()
  sh = ShardSet(d, o, torch.tensor([0, len(enc)], dtype=torch.int64).cuda(),
                torch.tensor([0, 1], dtype=torch.int64).cuda(), nbytes=len(data))
  ids, ntok, toff = pk.tokenize(sh)
  total = int(toff[len(enc)].item())
  assert total > pk.ids_estimate(len(data)) and ids.numel() >= total + 16
  oids, ontok = OracleTokenizer(VOCABS['bert']).run(data, off, 512, nthreads=4)
  assert np.array_equal(ntok.cpu().numpy()[:len(enc)], ontok)
  got = ids.cpu().numpy().view(np.uint16)[:total].astype(np.int64)
  assert np.array_equal(got, np.concatenate(compact(oids, ontok, off)).astype(np.int64))
  small = torch.empty(1000 + 16, dtype=torch.int16, device='cuda')
  with pytest.raises(CapacityError):
    pk.tok.tokenize_device(d, o, 512, out_ids=small, nbytes=len(data))


def test_tokenize_without_truncation_refuses_what_it_cannot_return(gpu):
  from lddl_amd.tokenizer import Tokenizer, TOKENS_MAX
  tok = Tokenizer(VOCABS['bert'])
  assert len(tok.tokenize('! ' * 600, truncation=False)) == 600
  with pytest.raises(ValueError):
    tok.tokenize('!' * (TOKENS_MAX + 10), truncation=False)


@pytest.mark.parametrize('seed', [0, 1])
def test_hip_tokenize_window_packing_edges(gpu, seed):
  """The scan's greedy 2 KiB windows: sentences whose lengths put the window
  end exactly at, just below and just past 2 KiB of the first sentence's
  16-B aligned start, at every start alignment; a sentence longer than a
  window (alone, to the serial path); runs of 40 one-word sentences (more
  than a window's 31); empty sentences between them"""
  from lddl_amd.synth import corpus_from_sentences
  from lddl_amd.tokenizer import Tokenizer
  rng = np.random.default_rng(seed)
  words = ['the', 'of', 'naïve', 'hello', 'electroencephalographically', '[SEP]', ',', 'x' * 120]

  def sent(nbytes):  # a sentence of exactly nbytes UTF-8 bytes
    out = ''
    while len(out.encode()) < nbytes - 4:
      out += words[int(rng.integers(0, len(words)))] + ' '
    out = out.encode()[:max(0, nbytes - 4)].decode('utf-8', 'ignore')
    return out + 'a' * (nbytes - len(out.encode()))
  sents = []
  for align in range(16):
    sents.append('z' * align)
    for target in (2032, 2040, 2047, 2048, 2049, 2064, 1024, 3000):
      a = int(rng.integers(1, target - 1))
      sents += [sent(a), sent(target - a), '']
    sents += ['w%d' % k for k in range(40)]
    sents += [sent(int(rng.integers(2040, 2100)))]
  tok = Tokenizer(VOCABS['bert'])
  c = corpus_from_sentences(sents, [0, len(sents)])
  ids, ntok = run_hip(tok, c.data, c.sent_off)
  oids, ontok = OracleTokenizer(VOCABS['bert']).run(c.data, c.sent_off, 512)
  assert np.array_equal(ntok, ontok)
  got, exp = compact(ids, ntok, c.sent_off), compact(oids, ontok, c.sent_off)
  bad = [i for i, (a, b) in enumerate(zip(got, exp)) if not np.array_equal(a, b)]
  assert not bad, bad[:10]


def test_algorithms_switched_on_one_ctx(gpu, monkeypatch):
  """Scratch reused across tokenizer algorithms on one ctx: the lane
  tokenizer (6, which allocates no finish scratch of its own) then the
  serial path (0) and the split tokenizer (5), whose finish pass reads
  pch / smeta / snslot / cnt8, then back -- every call identical to the
  oracle (the fault of round 5: the finish pass ran over scratch another
  algorithm had not allocated)"""
  from lddl_amd import synth
  from lddl_amd.tokenizer import Tokenizer
  c = synth.make_wiki(400_000, seed=41)
  oids, ontok = OracleTokenizer(VOCABS['bert']).run(c.data, c.sent_off, 512, nthreads=8)
  exp = compact(oids, ontok, c.sent_off)
  monkeypatch.setenv('LDDL_TOKENIZE_ALGO', '6')  # (the ctx builds the lane tokenizer's trie only when asked)
  tok = Tokenizer(VOCABS['bert'])
  for algo in (6, 0, 5, 6, 5, 0):
    assert tok.set_algo(algo) == algo
    ids, ntok = run_hip(tok, c.data, c.sent_off)
    assert np.array_equal(ntok, ontok), algo
    got = compact(ids, ntok, c.sent_off)
    assert all(np.array_equal(a.astype(np.int64), b.astype(np.int64)) for a, b in zip(got, exp)), algo
  with pytest.raises(Exception):
    tok.set_algo(3)
