"""Command-line front end: the reference's ``preprocess_bert_pretrain`` /
``preprocess_codebert_pretrain`` (lddl/dask/bert/pretrain.py:563-880,
pretrain_codebert.py) on MI355X.

Same flags, same input layout, same output files:

* input: ``--wikipedia <source>`` (reads ``<source>/<lang>/**.txt``),
  ``--books``, ``--common-crawl`` (``**.txt``), or ``--code`` (CodeBERT,
  ``**.txt`` of ``id<CODESPLIT>docstring<CODESPLIT>code`` records separated
  by ``\\r\\n``, readers.py:119-128); one document per non-empty stripped line
  as dask's read_text cuts lines (lddl_amd/readers.py), id = text up to the
  first whitespace, body = the rest after skipping one character
  (readers.py:142-147);
* partitions: one per input file, or per dask read_bytes block of each file
  with ``--block-size`` / ``--num-blocks`` (readers.py:43-57); CodeBERT: one
  per file (pretrain_codebert.py:479-485);
* output: ``--sink``/``part.{i}.parquet`` or ``part.{i}.parquet_{b}`` with
  the reference schema (lddl_amd/writer.py), ready for the load balancer
  (``python -m lddl_amd.balance``, load_balance.py); or, with
  ``--num-shards``, balanced straight away: the per-(partition, bin) row
  counts of every rank come from the packer through ONE all-gather (RCCL on
  the GPUs, ``balance.gather_bin_counts``) in place of the balancer's count
  pass over the files (load_balance.py:222-233), and each rank writes its
  ``shard-{k}.parquet[_b]`` files from the plan.

What runs where:
  host   an index of the input records (file, offset, length: integers
         only; with several ranks each indexes a share of the files and the
         shares are all-gathered) + --sample-ratio sampling + document
         shuffle over the index + partitioning of the shuffled records
         (equal bytes, fixed before the split like the reference's
         partitions) + reading and sentence-splitting ONLY this rank's
         records (NLTK Punkt when importable, pretrain.py:86; else a
         rule-based stand-in, see ``_rule_split``);
  GPU    tokenize -> pair packing -> binning -> materialisation -> string
         rendering (liblddl_amd.so), then the host parquet encoder.
  The rank's partitions stream through in chunks of --chunk-mb raw MB:
  --split-workers host processes (forked before the GPU is touched, so they
  hold the shuffled records copy-on-write and never see a GPU context) split
  the next chunks while chunk k is uploaded (pinned staging, async H2D),
  tokenised, packed and written.  Processes, not threads: the split is
  GIL-bound Python (Punkt or the stand-in) and would stall the main thread's
  GPU / writer calls.  The split time is reported separately
  (``host_split_s``) together with how much of it was hidden.

Determinism: the reference draws the sample, the document shuffle and every
partition's pairs from unseeded / dask-internal RNGs (pretrain.py:101-112,
readers.py:67-68), so no two runs of it agree.  Here all of them derive from
--seed: the sample and the shuffle from numpy's PCG64(seed), partition p's
pairs from random.seed(seed + p) exactly as the reference's
create_pairs_from_document would draw them after that seed.

Multi-GPU: launch under torch.distributed.run; rank r preprocesses the
contiguous partition range r of world (LPT would also do: partitions are
independent, pretrain.py:304,387) with no data-path collective.

Restart (``--resume``; the reference has none): after a chunk's
files are written, a marker ``<sink>/.lddl_done/chunk_<a>_<b>.json`` records
its files, per-(partition, bin) row counts and a key of every flag and input
file (name, size, mtime) the chunk's output depends on.  A rerun skips each
chunk whose marker carries the same key and whose files all exist; chunk
(a, b)'s output does not depend on the world size (partition p draws from
seed + p), so a restart may use another rank count.
"""
import argparse
import hashlib
import json
import os
import re
import sys
import time

import numpy as np

from . import synth


# ----------------------------------------------------------------- input --
from .readers import find_files_under, parse_str_of_num_bytes, estimate_block_size, count_partitions, \
    iter_lines, RecordIndex  # noqa: E402


def read_records(files, linedelimiter=None):
  """db.read_text + _filter_empty_strs (readers.py:30-31, 60-70): the
  stripped, non-empty lines of the files in order (lddl_amd/readers.py)."""
  for path in files:
    yield from iter_lines(path, linedelimiter)


def split_id_text(raw):
  """readers.py:142-147: id up to the first whitespace char, body after
  skipping exactly one character"""
  i = 0
  while i < len(raw) and not raw[i].isspace():
    i += 1
  return raw[:i], raw[i + 1:]


_ABBREV = frozenset('mr mrs ms dr prof sr jr st vs etc e.g i.e inc ltd co corp jan feb mar apr jun jul aug sep sept '
                    'oct nov dec no fig al approx dept est gen gov lt mt rev sgt u.s u.k'.split())
_CAND = re.compile(r'[.!?]+["\')\]]*\s+')


def _rule_split(text):
  """Rule-based stand-in for Punkt: a break after [.!?] (+ closing quotes /
  brackets) and whitespace when the next character starts a sentence and
  the word before is neither a known abbreviation nor a single-letter
  initial.  Not Punkt: the sentence boundaries are unpinned."""
  out, start = [], 0
  for m in _CAND.finditer(text):
    end = m.end()
    if end >= len(text):
      break
    nxt = text[end]
    if not (nxt.isupper() or nxt.isdigit() or nxt in '"\'([' ):
      continue
    prev = text[start:m.start()].rsplit(None, 1)
    w = prev[-1].lower().strip('("\'[') if prev else ''
    if m.group(0)[0] == '.' and (w in _ABBREV or (len(w) == 1 and w.isalpha())):
      continue
    out.append(text[start:m.end()])
    start = end
  out.append(text[start:])
  return out


def sentence_splitter(kind='auto'):
  """NLTK's sent_tokenize (the reference, pretrain.py:86) when importable
  with its punkt model, else the rule-based stand-in."""
  if kind in ('auto', 'punkt'):
    try:
      import nltk
      nltk.sent_tokenize('A b. C d.')
      return nltk.sent_tokenize, 'punkt'
    except Exception:
      if kind == 'punkt':
        raise RuntimeError('--sentence-splitter punkt: nltk / punkt not available')
  return _rule_split, 'rules'


def sample_order(n, seed, sample_ratio):
  """--sample-ratio sampling (readers.py:67-68) and the document shuffle
  (pretrain.py:101-112) over n records, both from PCG64(seed): the kept
  record indices in shuffled order."""
  rng = np.random.Generator(np.random.PCG64(seed))
  keep = np.arange(n, dtype=np.int64)
  if sample_ratio < 1.0:
    keep = keep[rng.random(n) < sample_ratio]
  return keep[rng.permutation(len(keep))]


def sample_shuffle(records, seed, sample_ratio):
  """sample_order over a list of records (tests, tools)."""
  records = list(records)
  return [records[i] for i in sample_order(len(records), seed, sample_ratio)]


def split_records(records, codebert=False, splitter=None):
  """Documents (in order) -> sentence-split synth.Corpus + doc ids; document
  i of the corpus is record i.

  BERT: _to_document (pretrain.py:82-97): sentences = split(body), each
  stripped, empty ones dropped.  CodeBERT: _to_code_pair
  (pretrain_codebert.py:126-159): docstring / code lines stripped, empty
  dropped; the doc's first doc_nseg_doc segments are its docstring."""
  sents, doc_off, nseg, ids = [], [0], [], []
  for r in records:
    if codebert:
      parts = r.split('<CODESPLIT>')
      if len(parts) != 3:
        raise ValueError('code record must have exactly 3 <CODESPLIT> parts (readers.py:150-151): %r' % r[:80])
      doc_id, docs, codes = synth.split_code_line(r)
      sents.extend(docs)
      sents.extend(codes)
      nseg.append(len(docs))
    else:
      doc_id, body = split_id_text(r)
      sents.extend(s.strip() for s in splitter(body) if s.strip())
    ids.append(doc_id)
    doc_off.append(len(sents))
  return synth.corpus_from_sentences(sents, doc_off, nseg if codebert else None), ids


def build_corpus(records, seed, sample_ratio, codebert=False, splitter=None):
  """sample_shuffle + split_records over the whole input (tests, tools)."""
  return split_records(sample_shuffle(records, seed, sample_ratio), codebert, splitter)


def partition_by_size(sizes, n_part):
  """Record offsets of n_part partitions of ~equal bytes over records of the
  given sizes (in order), documents kept whole."""
  sizes = np.asarray(sizes, dtype=np.int64)
  n = max(1, int(n_part))
  cum = np.concatenate([[0], np.cumsum(sizes)])
  cuts = np.searchsorted(cum, np.linspace(0, cum[-1], n + 1)[1:-1])
  off = np.concatenate([[0], cuts, [len(sizes)]]).astype(np.int64)
  return np.maximum.accumulate(off)


def partition_records(records, block_size=None, num_blocks=None):
  """--block-size / --num-blocks over a record list (tests, tools): ~equal
  byte partitions, num_blocks of them, or total / block_size."""
  if num_blocks is not None and block_size is not None:
    raise ValueError('Only one of num_blocks or blocksize needs to be set!')
  sizes = np.fromiter((len(r) for r in records), dtype=np.int64, count=len(records))
  if num_blocks is None:
    num_blocks = max(1, int(round(int(sizes.sum()) / block_size))) if block_size else 1
  return partition_by_size(sizes, min(num_blocks, max(1, len(records))))


def partition_docs(corpus, block_size=None, num_blocks=None):
  """--block-size / --num-blocks (readers.py:43-57): partitions of ~equal
  bytes, documents kept whole"""
  from .pipeline import partition_by_bytes
  if num_blocks is not None and block_size is not None:
    raise ValueError('Only one of num_blocks or blocksize needs to be set!')
  if num_blocks is None:
    num_blocks = max(1, int(round(corpus.nbytes / block_size))) if block_size else 1
  return partition_by_bytes(corpus, num_blocks)


# ------------------------------------------------------------------ CLI --
def attach_bool_arg(parser, flag_name, default=False, help_str=None):
  """--{flag} / --no-{flag} on one dest (lddl/utils.py:81-95)"""
  attr = flag_name.replace('-', '_')
  h = flag_name.replace('-', ' ') if help_str is None else help_str
  parser.add_argument('--{}'.format(flag_name), dest=attr, action='store_true', help=h)
  parser.add_argument('--no-{}'.format(flag_name), dest=attr, action='store_false', help=h)
  parser.set_defaults(**{attr: default})


def attach_args(parser=None, codebert=False):
  """The reference's flags (pretrain.py:618-880; pretrain_codebert.py's
  --code variant).  --schedule / --local-* are accepted for compatibility;
  this front end runs one process per GPU."""
  p = parser or argparse.ArgumentParser('lddl_amd preprocessor for the %s pretraining task'
                                        % ('CodeBERT' if codebert else 'BERT'))
  p.add_argument('--schedule', type=str, default='mpi', choices=['mpi', 'local'])
  p.add_argument('--local-n-workers', type=int, default=os.cpu_count())
  p.add_argument('--local-threads-per-worker', type=int, default=1)
  if codebert:
    p.add_argument('--code', type=str, default=None)
  else:
    p.add_argument('--wikipedia', type=str, default=None)
    p.add_argument('--books', type=str, default=None)
    p.add_argument('--common-crawl', type=str, default=None)
    p.add_argument('--wikipedia-lang', type=str, default='en')
  p.add_argument('--sink', type=str, required=True)
  p.add_argument('--output-format', type=str, default='parquet', choices=['parquet', 'txt'],
                 help='parquet (default) or txt, the reference\'s debugging text sink (pretrain.py:501-531): '
                      '{i}.txt / {i}_{b}.txt per partition (and bin)')
  p.add_argument('--target-seq-length', type=int, default=128)
  p.add_argument('--short-seq-prob', type=float, default=0.1)
  p.add_argument('--block-size', type=lambda x: parse_str_of_num_bytes(x, return_str=False), default=None,
                 help='n[KMG] bytes per dask block (lddl/download/utils.py:42-51)')
  p.add_argument('--num-blocks', type=int, default=None)
  p.add_argument('--bin-size', type=int, default=None)
  p.add_argument('--sample-ratio', type=float, default=0.9)
  p.add_argument('--seed', type=int, default=12345)
  p.add_argument('--duplicate-factor', type=int, default=1 if codebert else 5)
  p.add_argument('--vocab-file', type=str,
                 default=None, help='vocab.txt path (a local file: there is no hub access); default: the '
                 'bundled bert-base-uncased (BERT) or codebert_52000 (CodeBERT) vocab')
  attach_bool_arg(p, 'masking', default=False, help_str='static masking (pretrain.py:859-866)')
  p.add_argument('--masked-lm-ratio', type=float, default=0.15)
  p.add_argument('--sentence-splitter', type=str, default='auto', choices=['auto', 'punkt', 'rules'])
  p.add_argument('--chunk-mb', type=float, default=32.0,
                 help='raw MB of partitions per pipeline chunk (host split of the next chunks overlaps the GPU and '
                      'the writer on chunk k)')
  p.add_argument('--split-workers', type=int, default=None,
                 help='host processes splitting sentences ahead of the GPU (0: split inline; default: the cores '
                      'of this process\'s affinity (the reference\'s --local-n-workers defaults to os.cpu_count(), '
                      'pretrain.py:678) capped at LDDL_CPU_SHARE, default 16 -- one GPU\'s share of a GPU box, '
                      'beside the parquet encode threads')
  p.add_argument('--num-shards', type=int, default=None,
                 help='balance the output into this many shard-{k}.parquet[_b] files (balance_dask_output, '
                      'load_balance.py) with counts all-gathered from the packer')
  p.add_argument('--keep-orig', action='store_true', help='with --num-shards: keep the part files')
  p.add_argument('--resume', action='store_true',
                 help='write a completion marker per chunk and skip chunks an earlier run with the same flags '
                      'and inputs completed')
  return p


DONE_DIR = '.lddl_done'


def run_key(args, codebert, files, vocab, how, n_part):
  """Digest of everything a chunk's output depends on: the flags that reach
  the pipeline, the vocab and the input files (path, size, mtime)."""
  keys = ['target_seq_length', 'short_seq_prob', 'block_size', 'num_blocks', 'bin_size', 'sample_ratio', 'seed',
          'duplicate_factor', 'masking', 'masked_lm_ratio', 'output_format', 'wikipedia_lang']
  d = {k: getattr(args, k, None) for k in keys}
  d.update(codebert=codebert, splitter=how, n_part=n_part, vocab=os.path.abspath(vocab),
           vocab_size=os.path.getsize(vocab),
           files=[(os.path.abspath(f), os.path.getsize(f), os.stat(f).st_mtime_ns) for f in files])
  return hashlib.sha256(json.dumps(d, sort_keys=True).encode()).hexdigest()


def _marker(sink, a, b):
  return os.path.join(sink, DONE_DIR, 'chunk_%d_%d.json' % (a, b))


def load_marker(sink, a, b, key):
  """The marker of chunk [a, b) if it belongs to this run key and its files
  are all present, else None."""
  try:
    with open(_marker(sink, a, b)) as f:
      m = json.load(f)
  except (OSError, ValueError):
    return None
  if m.get('key') != key or not all(os.path.isfile(os.path.join(sink, f)) for f in m.get('files', [])):
    return None
  return m


def clear_markers(sink, a, b):
  """Remove every marker whose partition range overlaps [a, b): called before
  a chunk's files are (re)written, on every run with or without --resume, so
  no marker -- of this run key, an older one or other chunk bounds -- vouches
  for files that are about to change (a crash before save_marker then leaves
  the chunk without a marker)."""
  d = os.path.join(sink, DONE_DIR)
  try:
    names = os.listdir(d)
  except OSError:
    return
  for n in names:
    m = re.match(r'chunk_(\d+)_(\d+)\.json$', n)
    if m and int(m.group(1)) < b and a < int(m.group(2)):
      try:
        os.remove(os.path.join(d, n))
      except OSError:
        pass


def save_marker(sink, a, b, key, files, counts, n_pairs):
  """Written after the chunk's files (tmp + rename, so a crash leaves either
  no marker or a whole one)."""
  p = _marker(sink, a, b)
  os.makedirs(os.path.dirname(p), exist_ok=True)
  tmp = p + '.tmp%d' % os.getpid()
  with open(tmp, 'w') as f:
    json.dump({'key': key, 'files': sorted(os.path.relpath(x, sink) for x in files), 'counts': counts,
               'n_pairs': int(n_pairs)}, f)
  os.replace(tmp, p)


def _check(args):
  if args.output_format == 'txt' and getattr(args, 'num_shards', None):
    raise ValueError('--num-shards balances parquet shards; it does not apply to --output-format txt')
  if args.bin_size is not None:
    if args.bin_size > args.target_seq_length:
      raise ValueError('Please provide a bin size that is <= target-seq-length')
    if args.target_seq_length % args.bin_size != 0:
      raise ValueError('Please provide a bin size that can divide the target sequence length.')


_FE = {}  # the split workers' fork-inherited state (record index, order, mode, splitter)


def split_chunk(index, idx, codebert, split):
  """records idx of the index -> (corpus, doc ids): BERT records under the
  rule-based splitter go through the C splitter (splitnative: the same
  result as split_records, ~13x faster; LDDL_SPLIT_NATIVE=0 turns it off),
  everything else (CodeBERT, Punkt, a record that is not valid UTF-8, which
  the decode then reports) through split_records"""
  if not codebert and split is _rule_split and os.environ.get('LDDL_SPLIT_NATIVE', '1') != '0':
    from . import splitnative
    if splitnative.available():
      got = splitnative.split_raw(index.raws(idx))
      if got is not None:
        return got
  return split_records(index.texts(idx), codebert, split)


def _nice_worker():
  n = int(os.environ.get('LDDL_WORKER_NICE', '5'))
  if n > 0:
    try:
      os.nice(n)
    except OSError:
      pass


def _split_warm(_):
  return os.getpid()


def _split_worker(a, b):
  ts = time.perf_counter()
  corpus, ids = split_chunk(_FE['index'], _FE['order'][a:b], _FE['codebert'], _FE['split'])
  if _FE['codebert']:  # the writer's id column, built here in the worker, off the writer's path
    from .writer import str_array
    ids = str_array(ids)
  return corpus, ids, time.perf_counter() - ts


def chunk_pieces(part_end, lo, a, b, n):
  """partitions [a, b) cut into about n runs of ~equal bytes (whole
  partitions); part_end[p - lo] = bytes up to the end of partition p"""
  start = lambda q: int(part_end[q - 1 - lo]) if q > lo else 0
  if n <= 1 or b - a < 2:
    return [(a, b)]
  want = max(1, -(-(int(part_end[b - 1 - lo]) - start(a)) // n))
  out, s = [], a
  for q in range(a, b):
    if q + 1 == b or int(part_end[q - lo]) - start(s) >= want:
      out.append((s, q + 1))
      s = q + 1
  return out


def concat_corpora(corpora, ids):
  """one synth.Corpus and doc-id list / Arrow array of consecutive pieces"""
  if len(corpora) == 1:
    return corpora[0], ids[0]
  data = np.concatenate([c.data[c.sent_off[0]:c.sent_off[-1]] for c in corpora])
  so, dso = [np.zeros(1, np.int64)], [np.zeros(1, np.int64)]
  nb = ns = 0
  for c in corpora:
    so.append(c.sent_off[1:] - c.sent_off[0] + nb)
    dso.append(c.doc_sent_off[1:] - c.doc_sent_off[0] + ns)
    nb += c.nbytes
    ns += c.n_sent
  nseg = None
  if corpora[0].doc_nseg_doc is not None:
    nseg = np.concatenate([c.doc_nseg_doc for c in corpora])
  return synth.Corpus(data, np.concatenate(so), np.concatenate(dso), nseg), concat_ids(ids)


def concat_ids(ids):
  """the doc ids of consecutive pieces: lists (BERT) or Arrow arrays (CodeBERT)"""
  if len(ids) == 1:
    return ids[0]
  if isinstance(ids[0], list):
    return [x for i in ids for x in i]
  import pyarrow as pa
  return pa.concat_arrays(ids)


def input_files(args, codebert=False):
  """(files in the reference's bag order, line delimiter, source roots)"""
  if codebert:
    if not args.code:
      raise ValueError('--code is required')
    return find_files_under(args.code), '\r\n', [args.code]
  if not (args.wikipedia or args.books or args.common_crawl):
    raise ValueError('at least one of --wikipedia, --books and --common-crawl needs to be set')
  srcs = [os.path.join(args.wikipedia, args.wikipedia_lang) if args.wikipedia else None, args.books,
          args.common_crawl]
  # db.concat(bags) of read_wikipedia / read_books / read_common_crawl (pretrain.py:412-438)
  return [f for s in srcs if s for f in find_files_under(s)], None, [args.wikipedia, args.books, args.common_crawl]


def plan_input(args, codebert=False, rank=0, world=1, gloo=None):
  """The record index of the whole input, the sampled + shuffled record order
  and the partition offsets into it.  With several ranks each indexes every
  world-th file and the shares are all-gathered (host, gloo)."""
  files, delim, roots = input_files(args, codebert)
  if args.num_blocks is not None and args.block_size is not None:
    raise ValueError('Only one of num_blocks or blocksize needs to be set!')
  if codebert:  # read_code ignores the block flags: one partition per file (pretrain_codebert.py:479-485)
    n_part = len(files)
  else:
    bs = args.block_size
    if args.num_blocks is not None:
      bs = estimate_block_size(roots, args.num_blocks)  # readers.py:48-57 (the wikipedia ROOT, as the reference)
    n_part = count_partitions(files, bs)
  mine = set(range(rank, len(files), world))
  idx = RecordIndex.build(files, delim, file_ids=mine)
  if world > 1:
    import torch.distributed as dist
    parts = [None] * world
    dist.all_gather_object(parts, (idx.fid, idx.off, idx.len), group=gloo)
    idx = RecordIndex.merge(files, [RecordIndex(files, *p) for p in parts])
  order = sample_order(len(idx), args.seed, args.sample_ratio)
  pro = partition_by_size(idx.len[order], max(1, n_part))
  return idx, order, pro


def _dist_init(world):
  """One process per GPU (torch.distributed.run env): the default group on
  RCCL (nccl backend) for the count all-gather, a gloo group for host
  objects.  Returns the gloo group (None when single-process)."""
  if world <= 1:
    return None
  import torch
  import torch.distributed as dist
  if not dist.is_initialized():
    # LDDL_DIST_BACKEND=gloo: several ranks on one GPU (tests; RCCL needs a GPU per rank)
    backend = os.environ.get('LDDL_DIST_BACKEND') or ('nccl' if torch.cuda.is_available() else 'gloo')
    dist.init_process_group(backend)
  return dist.new_group(backend='gloo')


def main(args, codebert=False):
  """Returns (files written by this rank, timings dict)."""
  import torch
  from . import pipeline, writer, balance
  _check(args)
  rank = int(os.environ.get('RANK', 0))
  world = int(os.environ.get('WORLD_SIZE', 1))
  local = int(os.environ.get('LOCAL_RANK', 0))
  vocab = args.vocab_file or (pipeline.VOCAB_CODEBERT if codebert else pipeline.VOCAB_BERT)
  if not os.path.isfile(vocab):
    raise ValueError('--vocab-file must be a local vocab.txt (no hub access): %s' % vocab)
  t = {}
  wall0 = t0 = time.perf_counter()
  gloo = _dist_init(world)
  split, how = (None, 'code-lines') if codebert else sentence_splitter(args.sentence_splitter)
  index, order, pro = plan_input(args, codebert, rank, world, gloo)
  n_part = len(pro) - 1
  lo, hi = rank * n_part // world, (rank + 1) * n_part // world
  t['host_read_s'] = time.perf_counter() - t0
  # chunks of this rank's partitions, ~--chunk-mb raw MB each
  sizes = index.len[order[pro[lo]:pro[hi]]]
  cum = np.concatenate([[0], np.cumsum(sizes)])
  part_end = cum[pro[lo + 1:hi + 1] - pro[lo]]
  chunk_b = max(1, int(args.chunk_mb * (1 << 20)))
  bounds = [lo]
  acc0 = 0
  for p in range(lo, hi):
    if part_end[p - lo] - acc0 >= chunk_b and p + 1 < hi:
      bounds.append(p + 1)
      acc0 = part_end[p - lo]
  bounds.append(hi)
  chunks = [(a, b) for a, b in zip(bounds[:-1], bounds[1:]) if b > a]
  sink = os.path.abspath(os.path.expanduser(args.sink))
  nbins = args.target_seq_length // args.bin_size if args.bin_size else 1
  done, key = {}, None
  if args.resume:
    key = run_key(args, codebert, input_files(args, codebert)[0], vocab, how, n_part)
    for c, (a, b) in enumerate(chunks):
      m = load_marker(sink, a, b, key)
      if m is not None and np.asarray(m['counts']).shape == (b - a, nbins):
        done[c] = m
  todo = [c for c in range(len(chunks)) if c not in done]

  # the parquet encodes: a pool of processes forked first, before the GPU is
  # touched and before the split pool exists (a process forked beside a live
  # executor's threads can inherit their locks held; 16 forks beside 16 busy
  # split workers had also taken 0.17-0.29 s of the CPU share;
  # writer.ProcessEncoder; LDDL_ENCODE_PROCS=0: a thread pool)
  import concurrent.futures
  enc = None
  t0 = time.perf_counter()
  if args.output_format != 'txt':
    if os.environ.get('LDDL_ENCODE_PROCS', '1') != '0':
      enc = writer.ProcessEncoder()
    else:
      enc = concurrent.futures.ThreadPoolExecutor(writer.encode_workers())
  t['enc_start_s'] = time.perf_counter() - t0

  def close_enc():
    if enc is not None:
      enc.close() if isinstance(enc, writer.ProcessEncoder) else enc.shutdown(wait=False)

  # split workers: forked here, before anything touches the GPU; they read
  # their records from the index (integers only are inherited)
  sw = args.split_workers
  if sw is None:  # the host CPU share: affinity capped at LDDL_CPU_SHARE / 16 (hostinfo.cpu_share)
    from .hostinfo import cpu_share
    sw = cpu_share()
  # (a chunk's pieces are whole partitions: no more workers than partitions to split)
  n_todo = sum(chunks[c][1] - chunks[c][0] for c in todo)
  nw = min(max(0, sw), n_todo) if n_todo > 1 else 0
  pool = None
  if not codebert and split is _rule_split:
    from . import splitnative
    if splitnative.available():
      splitnative.props_table()  # (loaded here once; the forked workers share it)
  if nw > 0:
    import concurrent.futures
    import multiprocessing
    _FE.update(index=index, order=order, codebert=codebert, split=split)
    t0 = time.perf_counter()
    # (niced: the CPU share is shared with this process, whose thread drives
    # the GPU and the writer; LDDL_WORKER_NICE=0 keeps the default priority.
    # An executor, not multiprocessing.Pool: the Pool's handler threads poll
    # at 0.1 s, and its terminate / join took 0.12-0.25 s at the end)
    try:
      pool = concurrent.futures.ProcessPoolExecutor(nw, mp_context=multiprocessing.get_context('fork'),
                                                    initializer=_nice_worker)
      try:
        list(pool.map(_split_warm, range(nw)))  # (the first task forks every worker, while _FE holds the state)
      finally:
        _FE.clear()
    except BaseException:
      if pool is not None:
        pool.shutdown(wait=True, cancel_futures=True)
      close_enc()
      raise
    t['pool_start_s'] = time.perf_counter() - t0

  # a chunk is split as pieces of ~1/(2 nw) of it (whole partitions) on all
  # the workers at once: the GPU packs a chunk's partitions in parallel, one
  # wave each, so a chunk costs about one partition's latency and wants many
  # partitions, while its split should not wait on one worker
  def pieces(c):
    a, b = chunks[c]
    return chunk_pieces(part_end, lo, a, b, 2 * nw if pool is not None else 1)

  def submit(c):
    if pool is not None:
      return [pool.submit(_split_worker, int(pro[a]), int(pro[b])) for a, b in pieces(c)]
    ts = time.perf_counter()
    a, b = chunks[c]
    corpus, ids = split_chunk(index, order[int(pro[a]):int(pro[b])], codebert, split)

    class Done:
      def result(self):
        return corpus, ids, time.perf_counter() - ts
    return [Done()]

  def gather(fs):
    """the pieces of a chunk, in order: (corpora, doc ids, split seconds);
    pipeline.upload_pieces stages them for the GPU without a host concat"""
    got = [f_.result() for f_ in fs]
    return [g[0] for g in got], concat_ids([g[1] for g in got]), sum(g[2] for g in got)

  # the first chunks split while this process brings up the GPU context and
  # the device tables
  ahead = 2  # chunks split ahead of the GPU
  futs = {c: submit(c) for c in todo[:ahead]} if pool is not None else {}
  t0 = time.perf_counter()
  device = torch.device('cuda', local)
  try:
    torch.cuda.set_device(device)
    pk = pipeline.Packer(vocab, local, masking=args.masking and not codebert)
  except BaseException:
    if pool is not None:
      pool.shutdown(wait=True, cancel_futures=True)
    close_enc()
    raise
  t['gpu_init_s'] = time.perf_counter() - t0
  out = []
  counts = torch.zeros(hi - lo, nbins, dtype=torch.int64, device=device)  # rows per (partition, bin)
  t.update(host_split_s=0.0, split_wait_s=0.0, gpu_s=0.0, write_s=0.0, pairs=0, split_workers=nw,
           chunks_skipped=len(done))
  for c, m in done.items():
    a, b = chunks[c]
    counts[a - lo:b - lo] = torch.tensor(m['counts'], dtype=torch.int64)
    out += [os.path.join(sink, f) for f in m['files']]
    t['pairs'] += m['n_pairs']
  # parquet encodes of chunk k run on this pool while chunk k+1 splits,
  # uploads, tokenizes and packs; a chunk's --resume marker is saved once
  # all of its files are encoded (in chunk order)
  inflight = []  # (a, b, files, futures, counts, n_pairs) per chunk, oldest first

  def settle(keep):
    """finish the oldest chunks: those whose encodes are done, and while more
    than `keep` chunks are in flight, the oldest one (waiting for it)"""
    while inflight:
      if len(inflight) <= keep and not all(f_.done() for f_ in inflight[0][3]):
        break
      a_, b_, files_, futs_, cnt_, np_ = inflight.pop(0)
      tw_ = time.perf_counter()
      for f_ in futs_:
        f_.result()
      t['write_wait_s'] += time.perf_counter() - tw_
      if args.resume:
        save_marker(sink, a_, b_, key, files_, cnt_, np_)

  t['write_wait_s'] = 0.0
  try:
    for i, c in enumerate(todo):
      a, b = chunks[c]
      tw = time.perf_counter()
      corpus, ids, ts = gather(futs.pop(c) if c in futs else submit(c))
      t['split_wait_s'] += time.perf_counter() - tw
      t['host_split_s'] += ts
      if pool is not None and i + ahead < len(todo):
        futs[todo[i + ahead]] = submit(todo[i + ahead])  # overlaps this chunk's GPU work and parquet writes
      elif pool is not None and not futs and os.environ.get('LDDL_SPLIT_EARLY_EXIT', '1') != '0':
        # every split is in: the workers exit (0.2-0.4 s after a C2-size
        # run) beside the last chunks' GPU work and writes
        pool.shutdown(wait=False)
      t0 = time.perf_counter()
      sh = pipeline.upload_pieces(corpus, pro[a:b + 1] - pro[a], device)
      ids_d, ntok, toff = pk.tokenize(sh)
      # partition p packs after random.seed(args.seed + global p)
      res = pk.pack(sh, ids_d, ntok, toff, target_seq_length=args.target_seq_length, short_seq_prob=args.short_seq_prob,
                    duplicate_factor=args.duplicate_factor, seed=args.seed + a, bin_size=args.bin_size,
                    codebert=codebert, masking=args.masking and not codebert, masked_lm_ratio=args.masked_lm_ratio,
                    spans=True)
      counts[a - lo:b - lo] = res.bin_count.view(b - a, -1).to(torch.int64)
      torch.cuda.synchronize()
      t['gpu_s'] += time.perf_counter() - t0
      t0 = time.perf_counter()
      clear_markers(sink, a, b)
      kw = dict(bin_size=args.bin_size, codebert=codebert, masking=args.masking and not codebert, doc_ids=ids,
                part_base=a)
      cf = []
      if enc is None:
        wrote = writer.write_txt(pk, res, sink, **kw)
      else:
        wrote = writer.write_shards(pk, res, sink, executor=enc, pending=cf, **kw)
        for k_ in ('setup_s', 'render_s', 'table_s'):  # (the writer's stages: table_s = slot copies + hand-off)
          t['writer_' + k_] = t.get('writer_' + k_, 0.0) + writer.LAST_STATS.get(k_, 0.0)
      out += wrote
      inflight.append((a, b, wrote, cf, counts[a - lo:b - lo].tolist(), res.n_pairs))
      settle(2)  # at most two chunks' encodes behind the GPU
      t['write_s'] += time.perf_counter() - t0
      t['pairs'] += res.n_pairs
    t0 = time.perf_counter()
    settle(0)
    t['drain_s'] = time.perf_counter() - t0  # the last chunks' encodes
    if isinstance(enc, writer.ProcessEncoder):
      t['enc_slot_wait_s'], t['enc_copy_s'] = enc.wait_s, enc.copy_s
  finally:
    t0 = time.perf_counter()
    if pool is not None:
      pool.shutdown(wait=True, cancel_futures=True)
    t['teardown_split_s'] = time.perf_counter() - t0
    if enc is not None:
      enc.close() if isinstance(enc, writer.ProcessEncoder) else enc.shutdown(wait=True)
    index.close()
    t['teardown_s'] = time.perf_counter() - t0
    if getattr(enc, 'close_s', None):  # (absent when close() raised: that error propagates)
      t['teardown_enc_exit_s'], t['teardown_enc_unpin_s'], t['teardown_enc_rm_s'] = enc.close_s
  if args.num_shards:
    # balance_dask_output's job (load_balance.py:321-369) from the packer's
    # counts: one all-gather (RCCL) instead of its per-file count pass + MPI
    # Allreduce (:222-233); the plan is the same on every rank; shard k is
    # written by rank k % world from slices of the part files
    t0 = time.perf_counter()
    if world > 1:
      import torch.distributed as dist
      allc = balance.gather_bin_counts(counts if dist.get_backend() == 'nccl' else counts.cpu(), lo)
    else:
      allc = counts.cpu().numpy()
    shards, ns = balance.balance_counts(allc, args.num_shards, args.bin_size is not None, outdir=sink)
    written = balance.write_shards(shards, sink, rank, world)
    if world > 1:
      import torch.distributed as dist
      dist.barrier(group=gloo)
    if rank == 0:
      balance.store_num_samples(ns, sink)
      if not args.keep_orig:
        for p in out_all_parts(sink, allc.shape[0], nbins, args.bin_size is not None):
          if os.path.exists(p):
            os.remove(p)
        if args.resume:  # the markers name the part files just removed
          import shutil
          shutil.rmtree(os.path.join(sink, DONE_DIR), ignore_errors=True)
    t['balance_s'] = time.perf_counter() - t0
    t['shards'] = len(written)
    out = written
  t['wall_s'] = time.perf_counter() - wall0
  # the part of the host split hidden behind the GPU and the writer
  t['host_split_hidden_s'] = max(0.0, t['host_split_s'] - t['split_wait_s'])
  t.update(rank=rank, world=world, partitions=[lo, hi], documents=int(pro[hi] - pro[lo]), chunks=len(chunks),
           sentence_splitter=how, n_partitions=n_part)
  return out, t


def out_all_parts(sink, n_part, nbins, binned):
  """paths of every part file of the run"""
  if binned:
    return [os.path.join(sink, 'part.%d.parquet_%d' % (p, b)) for p in range(n_part) for b in range(nbins)]
  return [os.path.join(sink, 'part.%d.parquet' % p) for p in range(n_part)]


def console_script(argv=None, codebert=False):
  args = attach_args(codebert=codebert).parse_args(argv)
  tic = time.perf_counter()
  files, t = main(args, codebert)
  print('rank %d: %d files, %s' % (t['rank'], len(files), {k: v for k, v in t.items() if k != 'rank'}))
  print('Running the pipeline took {} s'.format(time.perf_counter() - tic))


def codebert_console_script(argv=None):
  console_script(argv, codebert=True)


if __name__ == '__main__':
  if len(sys.argv) > 1 and sys.argv[1] == 'codebert':
    codebert_console_script(sys.argv[2:])
  else:
    console_script()
