"""Synthetic corpora: the Books style and the
Wikipedia + Books mix behind BASELINE config C5."""
import numpy as np

from lddl_amd import synth


def test_books_style_shape():
  b = synth.make_books(2_000_000, seed=11)
  assert abs(b.nbytes - 2_000_000) < 0.3 * 2_000_000
  sents = [b.sentence(i) for i in range(b.n_sent)]  # valid UTF-8
  words = np.array([len(s.split()) for s in sents])
  assert 7 <= np.median(words) <= 16  # short sentences (median ~11 words)
  ndoc = np.diff(b.doc_sent_off)
  assert ndoc[:-1].min() >= 300  # books: long documents
  text = ' '.join(sents[:5000])
  for tok in ('"', "don't", "I'm", '—', 'Chapter'):
    assert tok in text, tok


def test_wikibooks_mixes_documents():
  m = synth.make_wikibooks(3_000_000, seed=5)
  w = synth.make_wiki(int(3_000_000 * 0.72), seed=5)
  b = synth.make_books(int(3_000_000 * 0.28), seed=6)
  assert m.n_doc == w.n_doc + b.n_doc and m.n_sent == w.n_sent + b.n_sent and m.nbytes == w.nbytes + b.nbytes
  lens = np.diff(m.doc_sent_off)
  books_at = np.nonzero(lens >= 300)[0]
  assert len(books_at) >= 1 and books_at.max() > 0  # book documents are not all at the front
  # the same documents, in another order
  docs = sorted(tuple(d) for d in m.documents())
  assert docs == sorted(tuple(d) for d in w.documents() + b.documents())
