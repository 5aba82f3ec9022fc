"""The CLI's sentence split in C (lddl_amd/splitnative.py, libsplit.so)
against the Python path it replaces (preprocess.split_records with the
rule-based splitter): identical sentences, document offsets and ids on
synthetic Wikipedia-style records and on adversarial ones (Unicode
whitespace, KELVIN SIGN abbreviations, dotted capital I, one-letter
initials, quotes and brackets, runs of punctuation, empty bodies, records
without a body), and invalid UTF-8 handed back to the Python path."""
import numpy as np
import pytest

from lddl_amd import build, preprocess, splitnative, synth


@pytest.fixture(scope='module', autouse=True)
def lib():
  build.build_split()
  assert splitnative.available()


def _py(records):
  return preprocess.split_records(records, False, preprocess._rule_split)


def _check(records):
  got = splitnative.split_raw([r.encode('utf-8') for r in records])
  assert got is not None
  exp = _py(records)
  gc, gi = got
  ec, ei = exp
  assert gi == ei
  assert np.array_equal(gc.doc_sent_off, ec.doc_sent_off)
  assert np.array_equal(gc.sent_off, ec.sent_off)
  assert bytes(gc.data) == bytes(ec.data)


def test_synthetic_wiki_records():
  c = synth.make_wiki(3_000_000, seed=4)
  docs = c.documents()
  records = ['wiki-%d %s' % (i, ' '.join(d)) for i, d in enumerate(docs)]
  _check(records)


ATOMS = ['Mr.', 'mr.', 'Dr.', 'U.S.', 'u.k.', 'e.g.', 'i.e.', 'etc.', 'U.K.', 'Ko.', 'A.', 'b.', 'İ.',
         'É.', 'Σ.', 'x.', 'Hello', 'world', 'The', 'the', '42', '٣', 'End.', 'Why?', 'Wow!', '?!',
         '...', '."', ".'", '.)', '.]', '("Hi', "'quoted'", '[x]', '(y)', ' ', ' ', '　', ' ',
         '\u0085', '\x1c', '\t', '\n', '  ', 'café', 'Ångström', '日本', '\U0001F600', 'ABC.',
         '.', '!', '?', 'Ⅲ', '½', '²']


def _adversarial(rng, n):
  out = []
  for i in range(n):
    k = int(rng.integers(0, 40))
    parts = []
    for _ in range(k):
      parts.append(ATOMS[int(rng.integers(0, len(ATOMS)))])
      parts.append([' ', '', ' ', '  ', ' '][int(rng.integers(0, 5))])
    body = ''.join(parts)
    sep = [' ', '\t', ' ', ' ', '　'][int(rng.integers(0, 5))]
    rid = ['doc%d' % i, 'dé%d' % i, '', 'x'][int(rng.integers(0, 4))]
    out.append(rid + sep + body if rng.random() < 0.95 else rid)
  return out


@pytest.mark.parametrize('seed', range(4))
def test_adversarial_records(seed):
  _check(_adversarial(np.random.default_rng(seed), 3000))


def test_edge_records():
  _check([])
  _check(['', ' ', 'id', 'id ', 'id  two', 'id A. B. C.', 'id Mr. Smith went. He left.', 'id K. Bob. x.',
          'id End. Next one.', 'id 3.14 is pi. 2 is two.', 'id "Quote." Next.', 'id a.b.c. D', 'id x. İs'])


def test_invalid_utf8_falls_back():
  assert splitnative.split_raw([b'ok A. B.', b'bad \xff\xfe. C.']) is None
  assert splitnative.split_raw([b'bad \xed\xa0\x80 surrogate']) is None
  assert splitnative.split_raw([b'trunc \xe2\x82']) is None


def test_random_code_points():
  """records of random code points drawn near the rules' decisions
  (sentence punctuation, closers, every whitespace, cased / digit / other
  letters from the whole range)"""
  rng = np.random.default_rng(11)
  pool = [c for c in range(0x110000) if not (0xD800 <= c <= 0xDFFF)]
  special = [ord(x) for x in '.!?"\')]([ '] + [c for c in range(0x110000) if chr(c).isspace()] + [0x212A, 0x130]
  recs = []
  for i in range(2000):
    n = int(rng.integers(0, 120))
    cps = [special[int(rng.integers(0, len(special)))] if rng.random() < 0.45 else
           (int(rng.integers(65, 123)) if rng.random() < 0.6 else pool[int(rng.integers(0, len(pool)))]) for _ in range(n)]
    recs.append(''.join(map(chr, cps)))
  _check(recs)


@pytest.mark.parametrize('crlf', [False, True])
def test_line_spans_match_numpy(crlf):
  """the C line scan (the record index's lines) against readers._line_spans
  on buffers dense in CR / LF / CR LF, with and without a final terminator"""
  from lddl_amd import readers
  rng = np.random.default_rng(int(crlf))
  for trial in range(300):
    n = int(rng.integers(0, 400))
    alphabet = np.array([10, 13, 65, 66, 32, 0xC2, 0xA0], dtype=np.uint8)
    p = np.array([0.15, 0.1, 0.4, 0.2, 0.1, 0.03, 0.02]) if trial % 3 else np.array([0.1, 0, 0.5, 0.3, 0.1, 0, 0])
    buf = rng.choice(alphabet, size=n, p=p / p.sum()).astype(np.uint8)
    got = splitnative.line_spans(buf, crlf)
    exp = readers._line_spans(buf, crlf)
    assert np.array_equal(got[0], exp[0]) and np.array_equal(got[1], exp[1]), (trial, bytes(buf))


@pytest.mark.parametrize('crlf', [False, True])
def test_line_spans_threaded_pieces(crlf):
  """the line index of a buffer cut into pieces after line terminators and
  indexed on threads equals the single pass: CR / LF / CR LF-dense buffers,
  tiny pieces (cuts land next to every kind of terminator), lines longer
  than a piece, no terminator at all"""
  from lddl_amd import readers
  rng = np.random.default_rng(10 + int(crlf))
  alphabet = np.array([10, 13, 65, 66, 32], dtype=np.uint8)
  for trial in range(200):
    n = int(rng.integers(0, 3000))
    p = [np.array([0.1, 0.1, 0.5, 0.2, 0.1]), np.array([0.005, 0.005, 0.6, 0.3, 0.09]),
         np.array([0, 0, 0.6, 0.3, 0.1])][trial % 3]
    buf = rng.choice(alphabet, size=n, p=p / p.sum()).astype(np.uint8)
    got = splitnative.line_spans(buf, crlf, threads=int(rng.integers(2, 9)), min_piece=int(rng.integers(1, 200)))
    exp = readers._line_spans(buf, crlf)
    assert np.array_equal(got[0], exp[0]) and np.array_equal(got[1], exp[1]), (trial, bytes(buf))
