"""Command-line front end: the reference's ``preprocess_bert_pretrain`` /
``preprocess_codebert_pretrain`` (lddl/dask/bert/pretrain.py:563-880,
pretrain_codebert.py) on MI355X.

Same flags, same input layout, same output files:

* input: ``--wikipedia <source>`` (reads ``<source>/<lang>/**.txt``),
  ``--books``, ``--common-crawl`` (``**.txt``), or ``--code`` (CodeBERT,
  ``**.txt`` of ``id<CODESPLIT>docstring<CODESPLIT>code`` records separated
  by ``\\r\\n``, readers.py:119-128); one document per non-empty stripped line
  (readers.py:30-31), id = text up to the first whitespace, body = the rest
  after skipping one character (readers.py:142-147);
* output: ``--sink``/``part.{i}.parquet`` or ``part.{i}.parquet_{b}`` with
  the reference schema (lddl_amd/writer.py), ready for the load balancer
  (``python -m lddl_amd.balance``, load_balance.py).

What runs where:
  host   read + --sample-ratio sampling + document shuffle + sentence split
         (NLTK Punkt when importable, pretrain.py:86; else a rule-based
         stand-in, see ``split_sentences``) + partitioning into
         --num-blocks / --block-size byte blocks (readers.py:48-57);
  GPU    tokenize -> pair packing -> binning -> materialisation -> string
         rendering (liblddl_amd.so), then the host parquet encoder.

Determinism: the reference draws the sample, the document shuffle and every
partition's pairs from unseeded / dask-internal RNGs (pretrain.py:101-112,
readers.py:67-68), so no two runs of it agree.  Here all of them derive from
--seed: the sample and the shuffle from numpy's PCG64(seed), partition p's
pairs from random.seed(seed + p) exactly as the reference's
create_pairs_from_document would draw them after that seed.

Multi-GPU: launch under torch.distributed.run; rank r preprocesses the
contiguous partition range r of world (LPT would also do: partitions are
independent, pretrain.py:304,387) with no data-path collective.
"""
import argparse
import os
import re
import sys
import time

import numpy as np

from . import synth


# ----------------------------------------------------------------- input --
def find_files_under(path, extensions=('.txt',)):
  """readers.py:34-40"""
  out = []
  for d, _, names in os.walk(path):
    out.extend(os.path.join(d, n) for n in names if os.path.splitext(n)[1] in extensions)
  return sorted(out)


def read_records(files, linedelimiter=None):
  """db.read_text + _filter_empty_strs (readers.py:30-31, 60-70): stripped,
  non-empty lines (records split on linedelimiter for code)."""
  for path in files:
    with open(path, encoding='utf-8', newline='' if linedelimiter else None) as f:
      text = f.read()
    parts = text.split(linedelimiter) if linedelimiter else text.splitlines()
    for s in parts:
      s = s.strip()
      if s:
        yield s


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


def build_corpus(records, seed, sample_ratio, codebert=False, splitter=None):
  """Documents (sampled, shuffled) -> sentence-split synth.Corpus + doc ids.

  BERT: _to_document (pretrain.py:82-97): sentences = split(body), each
  stripped, empty ones dropped.  CodeBERT: _to_code_pair
  (pretrain_codebert.py:126-159): docstring / code lines stripped, empty
  dropped; the doc's first doc_nseg_doc segments are its docstring."""
  rng = np.random.Generator(np.random.PCG64(seed))
  records = list(records)
  if sample_ratio < 1.0:
    keep = rng.random(len(records)) < sample_ratio
    records = [r for r, k in zip(records, keep) if k]
  order = rng.permutation(len(records))
  sents, doc_off, nseg, ids = [], [0], [], []
  for i in order:
    r = records[i]
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
  p.add_argument('--output-format', type=str, default='parquet', choices=['parquet'])
  p.add_argument('--target-seq-length', type=int, default=128)
  p.add_argument('--short-seq-prob', type=float, default=0.1)
  p.add_argument('--block-size', type=int, default=None)
  p.add_argument('--num-blocks', type=int, default=None)
  p.add_argument('--bin-size', type=int, default=None)
  p.add_argument('--sample-ratio', type=float, default=0.9)
  p.add_argument('--seed', type=int, default=12345)
  p.add_argument('--duplicate-factor', type=int, default=1 if codebert else 5)
  p.add_argument('--vocab-file', type=str,
                 default=None, help='vocab.txt path (a local file: there is no hub access); default: the '
                 'bundled bert-base-uncased (BERT) or codebert_52000 (CodeBERT) vocab')
  p.add_argument('--masking', action='store_true')
  p.add_argument('--masked-lm-ratio', type=float, default=0.15)
  p.add_argument('--sentence-splitter', type=str, default='auto', choices=['auto', 'punkt', 'rules'])
  return p


def _check(args):
  if args.bin_size is not None:
    if args.bin_size > args.target_seq_length:
      raise ValueError('Please provide a bin size that is <= target-seq-length')
    if args.target_seq_length % args.bin_size != 0:
      raise ValueError('Please provide a bin size that can divide the target sequence length.')


def main(args, codebert=False):
  """Returns (files written by this rank, timings dict)."""
  import torch
  from . import pipeline, writer
  _check(args)
  rank = int(os.environ.get('RANK', 0))
  world = int(os.environ.get('WORLD_SIZE', 1))
  local = int(os.environ.get('LOCAL_RANK', 0))
  vocab = args.vocab_file or (pipeline.VOCAB_CODEBERT if codebert else pipeline.VOCAB_BERT)
  if not os.path.isfile(vocab):
    raise ValueError('--vocab-file must be a local vocab.txt (no hub access): %s' % vocab)
  t = {}
  t0 = time.perf_counter()
  if codebert:
    if not args.code:
      raise ValueError('--code is required')
    files = find_files_under(args.code)
    recs = read_records(files, linedelimiter='\r\n')
    split, how = None, 'code-lines'
  else:
    srcs = [os.path.join(args.wikipedia, args.wikipedia_lang) if args.wikipedia else None, args.books,
            args.common_crawl]
    if not any(srcs):
      raise ValueError('at least one of --wikipedia, --books and --common-crawl needs to be set')
    files = [f for s in srcs if s for f in find_files_under(s)]
    recs = read_records(files)
    split, how = sentence_splitter(args.sentence_splitter)
  corpus, doc_ids = build_corpus(recs, args.seed, args.sample_ratio, codebert, split)
  pdo = partition_docs(corpus, args.block_size, args.num_blocks)
  n_part = len(pdo) - 1
  lo, hi = rank * n_part // world, (rank + 1) * n_part // world
  t['host_read_split_s'] = time.perf_counter() - t0
  # this rank's partitions as their own shard set (global partition ids kept)
  d0, d1 = int(pdo[lo]), int(pdo[hi])
  s0, s1 = int(corpus.doc_sent_off[d0]), int(corpus.doc_sent_off[d1])
  sub = synth.Corpus(corpus.data[corpus.sent_off[s0]:corpus.sent_off[s1]],
                     corpus.sent_off[s0:s1 + 1] - corpus.sent_off[s0], corpus.doc_sent_off[d0:d1 + 1] - s0,
                     None if corpus.doc_nseg_doc is None else corpus.doc_nseg_doc[d0:d1])
  device = torch.device('cuda', local)
  torch.cuda.set_device(device)
  t0 = time.perf_counter()
  pk = pipeline.Packer(vocab, local)
  sh = pipeline.upload(sub, pdo[lo:hi + 1] - d0, device)
  ids, ntok = pk.tokenize(sh)
  # partition p of this rank packs after random.seed(args.seed + global p)
  res = pk.pack(sh, ids, ntok, target_seq_length=args.target_seq_length, short_seq_prob=args.short_seq_prob,
                duplicate_factor=args.duplicate_factor, seed=args.seed + lo, bin_size=args.bin_size,
                codebert=codebert, masking=args.masking and not codebert, masked_lm_ratio=args.masked_lm_ratio)
  torch.cuda.synchronize()
  t['gpu_s'] = time.perf_counter() - t0
  t0 = time.perf_counter()
  sink = os.path.abspath(os.path.expanduser(args.sink))
  out = writer.write_shards(pk, res, sink, bin_size=args.bin_size, codebert=codebert,
                            masking=args.masking and not codebert, doc_ids=doc_ids[d0:d1], part_base=lo)
  t['write_s'] = time.perf_counter() - t0
  t.update(rank=rank, world=world, partitions=[lo, hi], documents=d1 - d0, pairs=res.n_pairs,
           sentence_splitter=how)
  return out, t


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
