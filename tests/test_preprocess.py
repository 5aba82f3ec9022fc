"""Host front end of the preprocessor CLI (no GPU): reader / id split /
sentence split / sampling / partitioning and the reference's flag defaults
(pretrain.py:618-880)."""
import os

import numpy as np
import pytest

from lddl_amd import preprocess


def test_split_id_text_matches_reference_rule():
  # readers.py:142-147: id to the first whitespace, skip exactly one char
  assert preprocess.split_id_text('wiki-1 Hello world.') == ('wiki-1', 'Hello world.')
  assert preprocess.split_id_text('wiki-2\t\tTwo tabs') == ('wiki-2', '\tTwo tabs')
  assert preprocess.split_id_text('only') == ('only', '')


def test_rule_splitter():
  s = preprocess._rule_split('Mr. Smith went to Washington. He arrived at 5 p.m. on Monday! Did he? Yes. '
                             'J. R. R. Tolkien wrote "The Hobbit." It sold well.')
  assert s[0] == 'Mr. Smith went to Washington. '
  assert [x.strip() for x in s[1:]] == ['He arrived at 5 p.m. on Monday!', 'Did he?', 'Yes.',
                                        'J. R. R. Tolkien wrote "The Hobbit."', 'It sold well.']
  assert preprocess._rule_split('no break here') == ['no break here']


def test_read_records_and_build_corpus(tmp_path):
  d = tmp_path / 'src' / 'en'
  d.mkdir(parents=True)
  (d / 'a.txt').write_text('wiki-1 First doc. Second sentence.\n\n   \nwiki-2 Another one here.\n')
  (d / 'b.txt').write_text('wiki-3 Third. Doc.\n')
  (d / 'skip.md').write_text('wiki-9 not read\n')
  files = preprocess.find_files_under(str(tmp_path / 'src' / 'en'))
  assert [os.path.basename(f) for f in files] == ['a.txt', 'b.txt']
  recs = list(preprocess.read_records(files))
  assert recs == ['wiki-1 First doc. Second sentence.', 'wiki-2 Another one here.', 'wiki-3 Third. Doc.']
  c, ids = preprocess.build_corpus(recs, 7, 1.0, splitter=preprocess._rule_split)
  assert sorted(ids) == ['wiki-1', 'wiki-2', 'wiki-3']
  docs = c.documents()
  byid = dict(zip(ids, docs))
  assert byid['wiki-1'] == ['First doc.', 'Second sentence.']
  assert byid['wiki-3'] == ['Third.', 'Doc.']
  # deterministic in the seed; sampling keeps ~ratio
  c2, ids2 = preprocess.build_corpus(recs, 7, 1.0, splitter=preprocess._rule_split)
  assert ids2 == ids and np.array_equal(c2.data, c.data)
  many = ['d%d x.' % i for i in range(2000)]
  _, kept = preprocess.build_corpus(many, 1, 0.9, splitter=preprocess._rule_split)
  assert 1700 < len(kept) < 1900


def test_code_records(tmp_path):
  (tmp_path / 'c.txt').write_bytes(b'py_0<CODESPLIT>Doc line\n  more<CODESPLIT>def f():\n    return 1\r\n'
                                   b'py_1<CODESPLIT><CODESPLIT>x = 1\r\n')
  recs = list(preprocess.read_records(preprocess.find_files_under(str(tmp_path)), linedelimiter='\r\n'))
  c, ids = preprocess.build_corpus(recs, 3, 1.0, codebert=True)
  docs = dict(zip(ids, c.documents()))
  nseg = dict(zip(ids, c.doc_nseg_doc.tolist()))
  assert docs['py_0'] == ['Doc line', 'more', 'def f():', 'return 1'] and nseg['py_0'] == 2
  assert docs['py_1'] == ['x = 1'] and nseg['py_1'] == 0


def test_flag_defaults_match_reference():
  a = preprocess.attach_args().parse_args(['--sink', 'x'])
  assert (a.schedule, a.target_seq_length, a.short_seq_prob, a.sample_ratio, a.seed, a.duplicate_factor,
          a.masked_lm_ratio, a.bin_size, a.block_size, a.num_blocks, a.wikipedia_lang, a.output_format) == (
              'mpi', 128, 0.1, 0.9, 12345, 5, 0.15, None, None, None, 'en', 'parquet')
  c = preprocess.attach_args(codebert=True).parse_args(['--sink', 'x', '--code', 'y'])
  assert c.duplicate_factor == 1


def test_partition_docs():
  from lddl_amd import synth
  c = synth.make_wiki(200_000, seed=3)
  pdo = preprocess.partition_docs(c, num_blocks=7)
  assert len(pdo) == 8 and pdo[0] == 0 and pdo[-1] == c.n_doc
  pdo = preprocess.partition_docs(c, block_size=50_000)
  assert len(pdo) - 1 == round(c.nbytes / 50_000)


def test_partition_records():
  recs = ['x' * (10 + (i * 37) % 200) for i in range(500)]
  pro = preprocess.partition_records(recs, num_blocks=7)
  assert len(pro) == 8 and pro[0] == 0 and pro[-1] == 500 and np.all(np.diff(pro) > 0)
  sizes = np.array([len(r) for r in recs])
  part = [sizes[pro[k]:pro[k + 1]].sum() for k in range(7)]
  assert max(part) - min(part) <= 2 * sizes.max()
  assert len(preprocess.partition_records(recs, block_size=10_000)) - 1 == round(sizes.sum() / 10_000)
  assert list(preprocess.partition_records(['a', 'b'], num_blocks=5)) == [0, 1, 2]
  with pytest.raises(ValueError):
    preprocess.partition_records(recs, block_size=10, num_blocks=2)


def test_build_corpus_is_shuffle_then_split():
  recs = ['wiki-%d Body %d here. Second one.' % (i, i) for i in range(50)]
  c, ids = preprocess.build_corpus(recs, 4, 0.8, splitter=preprocess._rule_split)
  c2, ids2 = preprocess.split_records(preprocess.sample_shuffle(recs, 4, 0.8), splitter=preprocess._rule_split)
  assert ids == ids2 and np.array_equal(c.data, c2.data) and np.array_equal(c.doc_sent_off, c2.doc_sent_off)
