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
  assert a.masking is False


def test_reference_full_flag_set_parses():
  """every flag of the reference's attach_args (pretrain.py:618-880), incl.
  attach_bool_arg's --masking / --no-masking pair (lddl/utils.py:81-95) and
  --output-format txt"""
  argv = ['--schedule', 'local', '--local-n-workers', '4', '--local-threads-per-worker', '1', '--wikipedia', 'w',
          '--books', 'b', '--common-crawl', 'c', '--sink', 's', '--output-format', 'txt', '--wikipedia-lang', 'en',
          '--target-seq-length', '512', '--short-seq-prob', '0.2', '--block-size', '64M', '--bin-size', '64',
          '--sample-ratio', '0.5', '--seed', '7', '--duplicate-factor', '3', '--vocab-file', 'v.txt', '--masking',
          '--masked-lm-ratio', '0.2']
  a = preprocess.attach_args().parse_args(argv)
  assert (a.output_format, a.masking, a.block_size, a.bin_size, a.masked_lm_ratio) == ('txt', True, 64 << 20, 64, 0.2)
  assert preprocess.attach_args().parse_args(argv + ['--no-masking']).masking is False
  assert preprocess.attach_args().parse_args(['--sink', 's', '--no-masking', '--masking']).masking is True
  a = preprocess.attach_args().parse_args(['--sink', 's', '--num-blocks', '4096'])
  assert a.num_blocks == 4096
  with pytest.raises(ValueError):
    preprocess._check(preprocess.attach_args().parse_args(['--sink', 's', '--output-format', 'txt',
                                                             '--num-shards', '4']))


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


# ---- reader semantics of db.read_text (readers.py:60-70) ----------------------
def _write(path, data):
  path.parent.mkdir(parents=True, exist_ok=True)
  path.write_bytes(data)
  return str(path)


def test_reader_breaks_lines_only_where_read_text_does(tmp_path):
  """read_text iterates a text-mode file: lines end at \\n, \\r\\n or \\r only.
  U+2028/2029, U+0085, \\v, \\f and \\x1c-\\x1e stay inside a record (str.splitlines
  would break there); str.strip() still removes them at the edges."""
  from lddl_amd import readers
  body = ('wiki-1 one still one and one\x85too\x0bv\x0cf\x1cx\x1dy\x1ez\n'
          'wiki-2 two\r\n'
          'wiki-3 three\rwiki-4 four\n'
          '   \n　 \n'
          '  wiki-5 padded \x85\x0c\n'
          'wiki-6 été no newline at end')
  f = _write(tmp_path / 'src' / 'a.txt', body.encode('utf-8'))
  want = ['wiki-1 one still one and one\x85too\x0bv\x0cf\x1cx\x1dy\x1ez', 'wiki-2 two', 'wiki-3 three',
          'wiki-4 four', 'wiki-5 padded', 'wiki-6 été no newline at end']
  assert list(readers.iter_lines(f)) == want
  idx = readers.RecordIndex.build([f])
  assert idx.texts(range(len(idx))) == want
  assert list(preprocess.read_records([f])) == want


def test_reader_code_records_split_on_crlf_only(tmp_path):
  from lddl_amd import readers
  f = _write(tmp_path / 'c.txt', b'py_0<CODESPLIT>doc\n more<CODESPLIT>x = 1\r\n  \r\npy_1<CODESPLIT>a\rb<CODESPLIT>y\r\n')
  want = ['py_0<CODESPLIT>doc\n more<CODESPLIT>x = 1', 'py_1<CODESPLIT>a\rb<CODESPLIT>y']
  assert list(readers.iter_lines(f, '\r\n')) == want
  idx = readers.RecordIndex.build([f], '\r\n')
  assert idx.texts(range(len(idx))) == want


@pytest.mark.parametrize('window', [None, 5, 37])
def test_reader_index_matches_text_mode_on_random_bytes(tmp_path, monkeypatch, window):
  """RecordIndex (vectorised, bytes) == Python text mode + strip + filter on
  random mixtures of terminators, ASCII / Unicode spaces and text, also with
  tiny file windows (cut after a line feed) that split runs every way."""
  from lddl_amd import readers
  if window:
    monkeypatch.setattr(readers, 'INDEX_WINDOW', window)
  rng = np.random.default_rng(3)
  atoms = ['a', 'bc', ' ', '\t', '\n', '\r', '\r\n', '\x0b', '\x0c', '\x1c', '\x1f', '\x85', '\xa0', ' ',
           '　', 'é', '中', '😀', '​', '\u2028', '\u1680', '\u205f', '\u3000', 'ア']
  for k in range(6):
    s = ''.join(atoms[i] for i in rng.integers(0, len(atoms), 3000))
    f = _write(tmp_path / ('r%d.txt' % k), s.encode('utf-8'))
    for d in (None, '\r\n'):
      idx = readers.RecordIndex.build([f], d)
      assert idx.texts(range(len(idx))) == list(readers.iter_lines(f, d)), (k, d)


def test_block_size_flag_and_partition_counts(tmp_path):
  from lddl_amd import readers
  assert readers.parse_str_of_num_bytes('128M') == 128 << 20
  assert readers.parse_str_of_num_bytes('2k') == 2048
  assert readers.parse_str_of_num_bytes('1000') == 100  # the reference drops a plain number's last digit
  with pytest.raises(ValueError):
    readers.parse_str_of_num_bytes('x')
  a = preprocess.attach_args().parse_args(['--sink', 'x', '--block-size', '64M'])
  assert a.block_size == 64 << 20
  # dask.bytes.read_bytes: max(1, size // blocksize) even blocks, none for an empty file
  assert [readers.dask_blocks(s, 100) for s in (0, 1, 99, 100, 199, 200, 250, 1000, 1050)] == [0, 1, 1, 1, 1, 2, 2, 10, 10]
  fs = [_write(tmp_path / 'w' / ('f%d.txt' % i), b'x y\n' * (10 + 40 * i)) for i in range(3)]
  assert readers.count_partitions(fs) == 3            # no block size: one partition per file
  assert readers.count_partitions(fs, 160) == sum(max(1, os.path.getsize(f) // 160) for f in fs)
  assert readers.estimate_block_size([str(tmp_path / 'w'), None], 4) == round(sum(map(os.path.getsize, fs)) / 4)


def test_default_partitions_are_one_per_input_file(tmp_path):
  """Without --num-blocks / --block-size the reference's read_text gives one
  partition per file (the previous front end made a single partition)."""
  for i in range(5):
    _write(tmp_path / 'src' / 'en' / ('wiki_%d.txt' % i),
           ''.join('wiki-%d-%d Some text here. More.\n' % (i, j) for j in range(20)).encode())
  args = preprocess.attach_args().parse_args(['--wikipedia', str(tmp_path / 'src'), '--sink', 'x'])
  idx, order, pro = preprocess.plan_input(args)
  assert len(pro) - 1 == 5
  assert len(idx) == 100 and 80 < len(order) < 100  # --sample-ratio 0.9
  args = preprocess.attach_args(codebert=True).parse_args(['--code', str(tmp_path / 'src'), '--sink', 'x',
                                                           '--num-blocks', '3'])
  _, _, pro = preprocess.plan_input(args, codebert=True)
  assert len(pro) - 1 == 5  # CodeBERT ignores the block flags (pretrain_codebert.py:479-485)


def _plan_worker(rank, world, root, port, q):
  import torch.distributed as dist
  os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
  dist.init_process_group('gloo', rank=rank, world_size=world)
  args = preprocess.attach_args().parse_args(['--wikipedia', root, '--sink', 'x', '--num-blocks', '7'])
  idx, order, pro = preprocess.plan_input(args, rank=rank, world=world, gloo=dist.group.WORLD)
  q.put((rank, idx.fid.tolist(), idx.off.tolist(), idx.len.tolist(), order.tolist(), pro.tolist()))
  dist.destroy_process_group()


def test_plan_input_sharded_over_ranks_matches_one_rank(tmp_path):
  """Each of 2 gloo ranks indexes half of the files; the all-gathered index,
  sample, shuffle and partitions equal the single-rank plan."""
  import socket
  import torch.multiprocessing as mp
  rng = np.random.default_rng(9)
  for i in range(7):
    _write(tmp_path / 'src' / 'en' / ('w%d.txt' % i),
           ''.join('wiki-%d-%d %s\n' % (i, j, 'word ' * int(rng.integers(1, 40))) for j in range(int(rng.integers(5, 60)))).encode())
  root = str(tmp_path / 'src')
  args = preprocess.attach_args().parse_args(['--wikipedia', root, '--sink', 'x', '--num-blocks', '7'])
  idx, order, pro = preprocess.plan_input(args)
  with socket.socket() as s:
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  ps = [ctx.Process(target=_plan_worker, args=(r, 2, root, port, q)) for r in range(2)]
  for p in ps:
    p.start()
  got = [q.get(timeout=120) for _ in ps]
  for p in ps:
    p.join(timeout=60)
  for _, fid, off, ln, od, pr in got:
    assert fid == idx.fid.tolist() and off == idx.off.tolist() and ln == idx.len.tolist()
    assert od == order.tolist() and pr == pro.tolist()


def test_resume_markers(tmp_path):
  """--resume: a chunk's marker is trusted only with the same run key and
  with all its files present; the key follows flags and input files"""
  src = tmp_path / 'wiki' / 'en'
  src.mkdir(parents=True)
  (src / 'a.txt').write_text('wiki-1 Hello there.\n')
  vocab = tmp_path / 'vocab.txt'
  vocab.write_text('[PAD]\n')
  sink = tmp_path / 'out'
  sink.mkdir()
  args = preprocess.attach_args().parse_args(['--wikipedia', str(tmp_path / 'wiki'), '--sink', str(sink), '--resume'])
  assert args.resume
  files = preprocess.input_files(args)[0]
  key = preprocess.run_key(args, False, files, str(vocab), 'rules', 1)
  assert key == preprocess.run_key(args, False, files, str(vocab), 'rules', 1)
  args2 = preprocess.attach_args().parse_args(['--wikipedia', str(tmp_path / 'wiki'), '--sink', str(sink),
                                               '--seed', '7'])
  assert preprocess.run_key(args2, False, files, str(vocab), 'rules', 1) != key
  assert preprocess.run_key(args, True, files, str(vocab), 'rules', 1) != key
  part = sink / 'part.0.parquet'
  part.write_bytes(b'x')
  assert preprocess.load_marker(str(sink), 0, 1, key) is None
  preprocess.save_marker(str(sink), 0, 1, key, [str(part)], [[3]], 3)
  m = preprocess.load_marker(str(sink), 0, 1, key)
  assert m == {'key': key, 'files': ['part.0.parquet'], 'counts': [[3]], 'n_pairs': 3}
  assert preprocess.load_marker(str(sink), 0, 1, 'other') is None
  assert preprocess.load_marker(str(sink), 0, 2, key) is None
  part.unlink()
  assert preprocess.load_marker(str(sink), 0, 1, key) is None
  # an input file that changed changes the key
  (src / 'a.txt').write_text('wiki-1 Hello there, again.\n')
  assert preprocess.run_key(args, False, files, str(vocab), 'rules', 1) != key


def test_clear_markers_removes_overlapping_chunks(tmp_path):
  """a chunk's markers (any run key, any chunk bounds overlapping it) go
  before its files are rewritten (a stale marker vouched for
  overwritten files)"""
  from lddl_amd import preprocess
  sink = str(tmp_path)
  for a, b in [(0, 4), (4, 8), (8, 12), (2, 6)]:
    preprocess.save_marker(sink, a, b, 'k', [], [[0]] * (b - a), 0)
  preprocess.clear_markers(sink, 4, 8)
  left = sorted(os.listdir(os.path.join(sink, preprocess.DONE_DIR)))
  assert left == ['chunk_0_4.json', 'chunk_8_12.json']
  assert preprocess.load_marker(sink, 0, 4, 'k') is not None
  preprocess.clear_markers(str(tmp_path / 'nothing'), 0, 1)  # no marker dir: no error


@pytest.mark.parametrize('codebert', [False, True])
def test_concat_corpora_equals_one_split(codebert):
  """a chunk split as pieces on several workers and concatenated is the
  chunk split at once"""
  from lddl_amd import synth, writer
  if codebert:
    recs = synth.make_code_lines(23, seed=3)
    split = None
  else:
    recs = ['wiki-%d %s' % (i, ' '.join(d)) for i, d in enumerate(synth.make_wiki(1 << 14, seed=5).documents())]
    split = preprocess.sentence_splitter('rules')[0]
  whole, ids = preprocess.split_records(recs, codebert, split)
  cuts = [0, 1, 1, len(recs) // 3, len(recs) - 1, len(recs)]
  parts = [preprocess.split_records(recs[a:b], codebert, split) for a, b in zip(cuts[:-1], cuts[1:])]
  pid = [writer.str_array(p[1]) for p in parts] if codebert else [p[1] for p in parts]
  got, gids = preprocess.concat_corpora([p[0] for p in parts], pid)
  assert bytes(got.data) == bytes(whole.data[:whole.nbytes])
  np.testing.assert_array_equal(got.sent_off, whole.sent_off)
  np.testing.assert_array_equal(got.doc_sent_off, whole.doc_sent_off)
  if codebert:
    np.testing.assert_array_equal(got.doc_nseg_doc, whole.doc_nseg_doc)
    assert gids.to_pylist() == ids
  else:
    assert got.doc_nseg_doc is None and gids == ids


def test_arrow_columns_without_pandas():
  """the writer's Arrow columns come from buffers (pa.array() imports pandas,
  ~0.5 s on the first call of a process)"""
  from lddl_amd import writer
  x = np.array([True, False, True, True, False, False, True, False, True])
  assert writer.np_array(x).to_pylist() == x.tolist()
  assert writer.np_array(x).slice(3, 5).to_pylist() == x[3:8].tolist()
  u = np.array([0, 7, 65535], np.uint16)
  assert writer.np_array(u).to_pylist() == u.tolist()
  assert writer.np_array(np.array([-3, 2**40], np.int64)).to_pylist() == [-3, 2**40]
  assert writer.str_array(['a', '', 'é☃']).to_pylist() == ['a', '', 'é☃']
  assert writer.str_array([]).to_pylist() == []


def test_chunk_pieces_cover_the_chunk():
  rng = np.random.default_rng(1)
  sizes = rng.integers(1, 1000, 40)
  part_end = np.cumsum(sizes)
  for lo, a, b, n in [(0, 0, 40, 8), (0, 5, 6, 8), (0, 3, 17, 1), (0, 0, 40, 100), (0, 10, 40, 3)]:
    pcs = preprocess.chunk_pieces(part_end[lo:], lo, a, b, n)
    assert pcs[0][0] == a and pcs[-1][1] == b
    assert all(x[1] == y[0] and x[0] < x[1] for x, y in zip(pcs, pcs[1:] + [(b, b + 1)]))
    assert len(pcs) <= max(1, n) + 1
  assert len(preprocess.chunk_pieces(np.full(32, 10).cumsum(), 0, 0, 32, 8)) == 8
  # a rank's range starting at lo > 0
  assert preprocess.chunk_pieces(np.full(10, 5).cumsum(), 7, 9, 17, 4) == [(9, 11), (11, 13), (13, 15), (15, 17)]


def test_batch_columns_past_32bit_offsets(monkeypatch):
  """a writer batch whose string bytes pass the 32-bit offset range is built
  with the large type and each file's slice cast back to the schema's"""
  import pyarrow as pa
  from lddl_amd import writer
  off = np.array([0, 3, 3, 7, 9], np.int64)
  data = np.frombuffer(b'abcdefghi', np.uint8)
  monkeypatch.setattr(writer, 'OFF32_LIMIT', 4)
  a = writer._arrow_rows(pa.string(), off, data, 4)
  assert a.type == pa.large_string()
  t = pa.Table.from_arrays([a], names=['A']).slice(1, 2).cast(pa.schema([('A', pa.string())]))
  assert t.schema.field('A').type == pa.string() and t.column('A').to_pylist() == ['', 'defg']
  monkeypatch.setattr(writer, 'OFF32_LIMIT', 2**31)
  assert writer._arrow_rows(pa.binary(), off, data, 4).type == pa.binary()


def test_file_table_rebases_offsets_past_2gib():
  """a writer batch whose string bytes really pass 2^31: the file
  after the 2 GiB row is rebuilt with offsets rebased to its first row, not
  sliced from the batch's large_string column (Arrow keeps a slice's absolute
  offsets, and the cast back to string rejects them).  np.zeros leaves the
  2 GiB buffer untouched: nothing reads its bytes."""
  import pyarrow as pa
  from lddl_amd import writer
  big = 2**31 + 5
  data = np.zeros(big + 3, np.uint8)
  data[big:] = np.frombuffer(b'xyz', np.uint8)
  off = np.array([0, big, big + 3], np.int64)
  sch = pa.schema([('A', pa.string()), ('num_tokens', pa.uint16())])
  raw = {'A': (pa.string(), off, data)}
  cols = {'A': writer._arrow_rows(pa.string(), off, data, 2), 'num_tokens': writer.np_array(np.array([7, 9], np.uint16))}
  assert cols['A'].type == pa.large_string()
  t = writer.file_table(sch, cols, raw, 1, 2)
  assert t.schema == sch
  assert t.column('A').to_pylist() == ['xyz'] and t.column('num_tokens').to_pylist() == [9]
  with pytest.raises(pa.ArrowInvalid):  # the old per-file slice + cast
    pa.Table.from_arrays([cols['A']], names=['A']).slice(1, 1).cast(pa.schema([('A', pa.string())]))
