"""Synthetic corpora for tests and bench.

There is no network here, so every corpus is synthetic.  Two styles:

* Wikipedia-style (``make_wiki``): documents of 3-60 sentences, sentence
  length lognormal (median 22 words, clipped to [3, 120]); words are 85 %
  Zipf(1.1) over alphabetic bert-base-uncased vocab entries, 10 % OOV
  composites of 2-4 vocab pieces (exercises ``##``), 3 % digits/punctuation,
  ~1 % accented Latin / Greek / CJK / Hangul / emoji / control / NBSP, plus
  rare >100-char words and literal ``[SEP]`` / ``[MASK]``.  Capitalised
  sentence starts.  Line format of the reference downloader
  (``lddl/download/wikipedia.py:58-63``): ``wiki-<id> <text>``.
* Books-style (``make_books``, BookCorpus as read by ``--books``,
  readers.py:88-99): long documents (300-3000 sentences) of short sentences
  (lognormal, median 11 words, clipped to [1, 80]); words as Wikipedia's but
  fewer OOV composites and ~14 % narrative tokens -- dialogue quotes and
  tags, contractions (``don't``, ``I'm``: apostrophes split as punctuation),
  em dashes, ellipses, chapter headings, character names.
  ``make_wikibooks`` mixes both at the documents' level (~72 % / 28 % of the
  bytes, English Wikipedia vs BookCorpus), as the reference's Wikipedia+Books
  runs shuffle them together (pretrain.py:100-111).
* Code-style (``make_code``): CodeSearchNet-like lines
  ``<lang>_<i><CODESPLIT><docstring><CODESPLIT><code>`` with 30 % empty
  docstrings and indented multi-line code
  (``shard_codebert_data.py:5,15-20``).

Both are emitted already sentence-split (the Punkt split is host work outside
the hot path): a ``Corpus`` holds the UTF-8 bytes
of every sentence back to back, ``sent_off`` (int64, n_sent+1) and
``doc_sent_off`` (int64, n_doc+1).
"""
from __future__ import annotations

import dataclasses
import os
import re

import numpy as np

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data')


@dataclasses.dataclass
class Corpus:
  data: np.ndarray          # uint8 [nbytes]
  sent_off: np.ndarray      # int64 [n_sent + 1]
  doc_sent_off: np.ndarray  # int64 [n_doc + 1]
  # CodeBERT only: per doc, number of docstring segments (the first ones)
  doc_nseg_doc: np.ndarray | None = None

  @property
  def n_sent(self):
    return len(self.sent_off) - 1

  @property
  def n_doc(self):
    return len(self.doc_sent_off) - 1

  @property
  def nbytes(self):
    return int(self.sent_off[-1] - self.sent_off[0])

  def sentence(self, i) -> str:
    return bytes(self.data[self.sent_off[i]:self.sent_off[i + 1]]).decode('utf-8')

  def documents(self):
    """list[list[str]] (slow; tests only)."""
    return [[self.sentence(s) for s in range(self.doc_sent_off[d], self.doc_sent_off[d + 1])]
            for d in range(self.n_doc)]


def _load_vocab(path):
  with open(path, encoding='utf-8') as f:
    return [l.rstrip('\n') for l in f]


_EXOTIC = [
    'café', 'naïve', 'Müller', 'Ångström', 'façade', 'São', 'Dvořák', 'İstanbul', 'Łódź',
    'Σοφία', 'ΣΑΣ', 'λόγος', '東京', '中文字', '한국어', '서울', '😀', '🚀ok', 'éte',
    'a\u0007b', 'x​y', 'foo bar', 'ﬁne', 'Ⅻ', 'ｆｕｌｌ', 'ß', 'ǅemal', '𝐛𝐨𝐥𝐝',
    'a☃b', 'm̀́̂', 'tab\there', 'русский', 'العربية', 'हिन्दी',
]
_PUNCT = ['1985', '3.14', '42', '2,000', '(', ')', '-', '—', '"', "'", ';', ':', '%', '$5',
          '&', '/', '[1]', 'e.g.', '#', '@user', '...', '$$', '<b>', '~', '`x`']


def _build_pool(vocab, rng, n_oov=20000):
  alpha = [w for w in vocab if re.fullmatch(r'[a-z]+', w)]
  # the vocab lists single letters before whole words; keep 'a'/'i' as words
  alpha = [w for w in alpha if len(w) > 1 or w in ('a', 'i')] + \
          [w for w in alpha if len(w) == 1 and w not in ('a', 'i')]
  pieces = [w[2:] for w in vocab if re.fullmatch(r'##[a-z]+', w)]
  oov = []
  for _ in range(n_oov):
    k = int(rng.integers(2, 5))
    w = alpha[int(rng.integers(0, len(alpha)))]
    for _ in range(k - 1):
      w += pieces[int(rng.integers(0, len(pieces)))]
    oov.append(w)
  return alpha, oov


_NARRATIVE = ['"', '"', "'", "I'm", "don't", "can't", "it's", "you're", "he'd", "she'll", "won't", "'s",
              "didn't", "I'll", "we're", "they'd", "ain't", "y'all", '—', '…', '...', 'Mr.', 'Mrs.', 'Dr.',
              '" he said', '" she whispered', '," I asked', '?"', '!"', 'Chapter', 'CHAPTER', 'Prologue',
              'Harry', 'Elizabeth', 'Darcy', 'Jonah', 'Kaelen', 'okay', 'yeah', 'Oh', 'gonna', 'wanna', '?!',
              'Hmm', 'Shh', 'Mom', 'Dad']


class _WordTable:
  """Byte pool of words + per-category index ranges and sampling weights."""

  def __init__(self, vocab, rng, books=False):
    alpha, oov = _build_pool(vocab, rng)
    longw = [''.join(chr(97 + int(c)) for c in rng.integers(0, 26, int(n)))
             for n in rng.integers(101, 160, 16)]
    cats = [alpha, oov, _PUNCT, _EXOTIC, longw, ['[SEP]', '[MASK]']]
    if books:
      cats.append(_NARRATIVE)
    self.words = [w for c in cats for w in c]
    enc = [w.encode('utf-8') for w in self.words]
    self.wlen = np.array([len(b) for b in enc], dtype=np.int64)
    self.woff = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum(self.wlen, out=self.woff[1:])
    self.pool = np.frombuffer(b''.join(enc), dtype=np.uint8)
    bases = np.cumsum([0] + [len(c) for c in cats])
    self.cat_base = bases[:-1]
    self.cat_size = np.array([len(c) for c in cats])
    if books:
      self.cat_p = np.array([0.80, 0.04, 0.018, 0.002, 1e-6, 1e-7, 0.14])
    else:
      self.cat_p = np.array([0.85, 0.10, 0.03, 0.0099889, 1e-5, 1e-6])
    self.cat_p /= self.cat_p.sum()
    r = np.arange(1, len(alpha) + 1, dtype=np.float64)
    z = r ** -1.1
    self.zipf_cdf = np.cumsum(z / z.sum())
    # is the first byte an ASCII lowercase letter (capitalisable)?
    self.first = self.pool[self.woff[:-1]]

  def sample(self, rng, n):
    cat = rng.choice(len(self.cat_p), size=n, p=self.cat_p)
    u = rng.random(n)
    idx = (u * self.cat_size[cat]).astype(np.int64)
    zipf = np.searchsorted(self.zipf_cdf, u[cat == 0])
    idx[cat == 0] = np.minimum(zipf, self.cat_size[0] - 1)
    return self.cat_base[cat] + idx


def _assemble(pool, src_off, lens):
  """Concatenate pool[src_off[i]:src_off[i]+lens[i]] for all i (vectorised)."""
  total = int(lens.sum())
  dst = np.zeros(len(lens) + 1, dtype=np.int64)
  np.cumsum(lens, out=dst[1:])
  idx = np.arange(total, dtype=np.int64)
  idx += np.repeat(src_off - dst[:-1], lens)
  return pool[idx], dst


def make_wiki(target_bytes, seed=20261015, vocab_path=None):
  """Wikipedia-style sentence-split corpus of about ``target_bytes`` bytes."""
  return _make_prose(target_bytes, seed, vocab_path, books=False)


def make_books(target_bytes, seed=20261015, vocab_path=None):
  """Books-style (BookCorpus) sentence-split corpus of about ``target_bytes``."""
  return _make_prose(target_bytes, seed, vocab_path, books=True)


def make_wikibooks(target_bytes, seed=20261015, vocab_path=None, books_frac=0.28):
  """Wikipedia + Books: both styles, documents interleaved in a random order."""
  w = make_wiki(int(target_bytes * (1 - books_frac)), seed, vocab_path)
  b = make_books(int(target_bytes * books_frac), seed + 1, vocab_path)
  return interleave_documents([w, b], np.random.default_rng(seed + 2))


def interleave_documents(corpora, rng):
  """One corpus of every document of the given corpora in a random order."""
  spans, nsent = [], []  # (corpus, doc) byte spans and sentence counts
  datas = [c.data[c.sent_off[0]:c.sent_off[-1]] for c in corpora]
  base = np.cumsum([0] + [len(d) for d in datas])
  pool = np.concatenate(datas) if datas else np.zeros(0, np.uint8)
  d_beg, d_len, s_lens = [], [], []
  for k, c in enumerate(corpora):
    so = c.sent_off - c.sent_off[0]
    d_beg.append(base[k] + so[c.doc_sent_off[:-1]])
    d_len.append(so[c.doc_sent_off[1:]] - so[c.doc_sent_off[:-1]])
    s_lens.append([np.diff(so[c.doc_sent_off[d]:c.doc_sent_off[d + 1] + 1]) for d in range(c.n_doc)])
  d_beg, d_len = np.concatenate(d_beg), np.concatenate(d_len)
  s_all = [x for sl in s_lens for x in sl]
  order = rng.permutation(len(d_beg))
  data, _ = _assemble(pool, d_beg[order], d_len[order])
  sl = np.concatenate([s_all[i] for i in order]) if len(order) else np.zeros(0, np.int64)
  sent_off = np.concatenate([[0], np.cumsum(sl)]).astype(np.int64)
  doc_sent_off = np.concatenate([[0], np.cumsum([len(s_all[i]) for i in order])]).astype(np.int64)
  del spans, nsent
  return Corpus(data, sent_off, doc_sent_off)


def _make_prose(target_bytes, seed, vocab_path, books):
  rng = np.random.default_rng(seed)
  vocab = _load_vocab(vocab_path or os.path.join(DATA_DIR, 'bert_vocab.txt'))
  table = _WordTable(vocab, rng, books=books)
  avg_word = 5.0 if books else 6.2
  n_words = max(64, int(target_bytes / avg_word))
  # sentence lengths (words) and document sizes (sentences)
  med, sig, lo, hi = (11.0, 0.65, 1, 80) if books else (22.0, 0.55, 3, 120)
  n_sent_est = int(n_words // med) + 8
  slen = np.clip(np.rint(rng.lognormal(np.log(med), sig, n_sent_est)), lo, hi).astype(np.int64)
  csum = np.cumsum(slen)
  n_sent = int(np.searchsorted(csum, n_words)) + 1
  n_sent = min(n_sent, len(slen))
  slen = slen[:n_sent]
  n_words = int(slen.sum())
  w = table.sample(rng, n_words)
  wl = table.wlen[w]
  # separators: ' ' between words, ',' sometimes, '.' (or ?/!) at sentence end
  sent_last = np.cumsum(slen) - 1
  sent_first = sent_last - slen + 1
  sep = np.full(n_words, ord(' '), dtype=np.uint8)
  comma = rng.random(n_words) < 0.06
  end = np.zeros(n_words, dtype=bool)
  end[sent_last] = True
  # each word emits: bytes, optional ',' , then ' ' (except sentence end: '.')
  extra = np.where(end, 1, np.where(comma, 2, 1)).astype(np.int64)
  # build word bytes
  wb, wdst = _assemble(table.pool, table.woff[w], wl)
  # capitalise sentence starts
  fb = wdst[sent_first]
  isl = (wb[fb] >= 97) & (wb[fb] <= 122)
  wb[fb[isl]] -= 32
  # interleave separators: final layout per word = wordbytes + extra bytes
  tot = wl + extra
  dst = np.zeros(n_words + 1, dtype=np.int64)
  np.cumsum(tot, out=dst[1:])
  out = np.empty(int(dst[-1]), dtype=np.uint8)
  # word bytes
  idx = np.arange(len(wb), dtype=np.int64) + np.repeat(dst[:-1] - wdst[:-1], wl)
  out[idx] = wb
  p0 = dst[:-1] + wl
  endc = np.full(n_words, ord('.'), dtype=np.uint8)
  q = rng.random(n_words)
  endc[q < 0.05] = ord('?')
  endc[(q >= 0.05) & (q < 0.08)] = ord('!')
  out[p0] = np.where(end, endc, np.where(comma, ord(','), sep))
  out[p0[comma & ~end] + 1] = ord(' ')
  # sentence byte offsets: sentences end after their terminator; the ' '
  # between sentences is dropped (sentences are stripped, pretrain.py:86)
  sent_end = dst[sent_last + 1]
  sent_beg = dst[sent_first]
  sent_off = np.empty(n_sent + 1, dtype=np.int64)
  sent_off[:-1] = sent_beg
  sent_off[-1] = sent_end[-1]
  assert np.all(sent_off[1:] == sent_end)
  # documents: 3-60 sentences (an article), 300-3000 (a book)
  dl = rng.integers(300, 3001, n_sent // 300 + 2) if books else rng.integers(3, 61, n_sent // 3 + 2)
  dcs = np.cumsum(dl)
  n_doc = int(np.searchsorted(dcs, n_sent)) + 1
  doc_sent_off = np.concatenate([[0], np.minimum(dcs[:n_doc], n_sent)]).astype(np.int64)
  return Corpus(out, sent_off, doc_sent_off)


_IDENTS = ['self', 'data', 'value', 'result', 'items', 'config', 'index', 'count', 'name', 'path',
           'buffer', 'offset', 'parse', 'get', 'set', 'update', 'load', 'save', 'user', 'request',
           'response', 'client', 'server', 'node', 'tree', 'list', 'dict', 'key', 'token', 'model']
_KW = ['def', 'return', 'if', 'else', 'for', 'in', 'while', 'import', 'from', 'class', 'not',
       'and', 'or', 'None', 'True', 'False', 'try', 'except', 'raise', 'with', 'as', 'lambda']
_OPS = ['=', '==', '+', '-', '*', '/', '(', ')', '[', ']', '{', '}', ':', ',', '.', '+=', '!=',
        '<', '>', '->', '**', '%']


def _ident(rng):
  k = int(rng.integers(1, 4))
  parts = [_IDENTS[int(rng.integers(0, len(_IDENTS)))] for _ in range(k)]
  if rng.random() < 0.3:
    return parts[0] + ''.join(p.capitalize() for p in parts[1:])
  return '_'.join(parts)


def make_code_lines(n_lines, seed=20261015):
  """CodeSearchNet-style raw lines (python-ish), ``id<CODESPLIT>doc<CODESPLIT>code``."""
  rng = np.random.default_rng(seed)
  lines = []
  for i in range(n_lines):
    if rng.random() < 0.3:
      doc = ''
    else:
      nd = int(rng.integers(1, 5))
      doc = '\n'.join(' '.join(_ident(rng).replace('_', ' ') for _ in range(int(rng.integers(3, 14))))
                      for _ in range(nd))
    nl = int(rng.integers(3, 61))
    code = ['def %s(%s):' % (_ident(rng), ', '.join(_ident(rng) for _ in range(int(rng.integers(0, 4)))))]
    for _ in range(nl - 1):
      ind = '    ' * int(rng.integers(1, 4))
      toks = []
      for _ in range(int(rng.integers(2, 12))):
        r = rng.random()
        if r < 0.5:
          toks.append(_ident(rng))
        elif r < 0.7:
          toks.append(_KW[int(rng.integers(0, len(_KW)))])
        elif r < 0.9:
          toks.append(_OPS[int(rng.integers(0, len(_OPS)))])
        else:
          toks.append(str(int(rng.integers(0, 10000))))
      code.append(ind + ' '.join(toks))
    lines.append('python_%d<CODESPLIT>%s<CODESPLIT>%s' % (i, doc, '\n'.join(code)))
  return lines


def split_code_line(line):
  """Reference ``_to_code_pair`` split (pretrain_codebert.py:126-141,
  readers.py:150-151): returns (id, doc_segments, code_segments) as str."""
  parts = line.split('<CODESPLIT>')
  code_pair_id, docstring, code = parts  # must be exactly 3 parts
  docs = [s.strip() for s in docstring.split('\n')]
  codes = [s.strip() for s in code.split('\n')]
  return code_pair_id, [s for s in docs if s], [s for s in codes if s]


def make_code(n_lines, seed=20261015):
  """Code corpus, sentence-split: per doc, docstring segments then code segments."""
  sents = []
  doc_off = [0]
  ndoc = []
  for line in make_code_lines(n_lines, seed):
    _, docs, codes = split_code_line(line)
    sents.extend(docs)
    sents.extend(codes)
    doc_off.append(len(sents))
    ndoc.append(len(docs))
  return corpus_from_sentences(sents, doc_off, ndoc)


def corpus_from_sentences(sents, doc_sent_off, doc_nseg_doc=None):
  enc = [s.encode('utf-8') for s in sents]
  off = np.zeros(len(enc) + 1, dtype=np.int64)
  np.cumsum([len(b) for b in enc], out=off[1:])
  data = np.frombuffer(b''.join(enc), dtype=np.uint8).copy() if enc else np.zeros(0, np.uint8)
  return Corpus(data, off, np.asarray(doc_sent_off, dtype=np.int64),
                None if doc_nseg_doc is None else np.asarray(doc_nseg_doc, dtype=np.int32))


def corpus_from_documents(docs):
  sents = [s for d in docs for s in d]
  off = np.zeros(len(docs) + 1, dtype=np.int64)
  np.cumsum([len(d) for d in docs], out=off[1:])
  return corpus_from_sentences(sents, off)
