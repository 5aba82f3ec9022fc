"""ORACLE -- test infrastructure only (tests/, __graft_entry__.smoke(),
bench.py cpu_baseline).  Never imported by lddl_amd/.

Pure-Python restatement of the reference's pair packing, driven by CPython's
own ``random`` module (MT19937, the RNG the reference uses):

  * ``bert_pairs``      lddl/dask/bert/pretrain.py:241-365
                        create_pairs_from_document (+ _truncate_seq_pair :161-176)
  * ``codebert_pairs``  lddl/dask/bert/pretrain_codebert.py:343-442
                        create_pairs_from_document (+ _truncate_seq :236-247)
  * ``masked_lm``       pretrain.py:182-238 create_masked_lm_predictions
                        (static masking, --masking; vocab_words = the vocab
                        file's tokens in file order, i.e. token id = index)
  * ``partition_pairs`` pretrain.py:386-402 / pretrain_codebert.py:460-477
                        _to_partition_pairs: duplicate_factor passes over the
                        partition's documents, then random.shuffle
  * ``bin_of`` / ``binned_order``  binning.py:63-93 _to_dataframe_binned:
                        bin = (num_tokens-1)//bin_size clamped to nbins-1,
                        stable per-bin grouping of the shuffled rows

Seeding (the reference's partition RNG is unseeded): partition
p of a run with --seed S is packed after ``random.seed(S + p)``.
Documents are lists of sentences; a sentence is a list of token ids.  Empty
sentences and documents are dropped first (pretrain.py:89-97).

Pinned against the reference itself by tests/golden/pack_*.json, produced by
tools/gen_golden_pack.py from the imported reference functions.
"""
import random

import numpy as np


def _truncate_seq_pair(a, b, max_num_tokens, rnd):
  # pretrain.py:161-176; a, b are [front, back) windows [lo, hi] as lists
  while True:
    la, lb = a[1] - a[0], b[1] - b[0]
    if la + lb <= max_num_tokens:
      break
    t = a if la > lb else b
    assert t[1] - t[0] >= 1
    if rnd.random() < 0.5:
      t[0] += 1
    else:
      t[1] -= 1


def masked_lm(tokens_a, tokens_b, ratio, n_vocab, cls_id, sep_id, mask_id, rnd):
  """create_masked_lm_predictions over token ids -> (A', B', positions, labels)."""
  tokens = [cls_id] + list(tokens_a) + [sep_id] + list(tokens_b) + [sep_id]
  cand = [i for i, t in enumerate(tokens) if t != cls_id and t != sep_id]
  rnd.shuffle(cand)
  out = list(tokens)
  num_to_predict = max(1, int(round(len(tokens) * ratio)))
  picked = []
  for index in cand:
    if len(picked) >= num_to_predict:
      break
    if rnd.random() < 0.8:
      new = mask_id
    elif rnd.random() < 0.5:
      new = tokens[index]
    else:
      new = rnd.randint(0, n_vocab - 1)
    out[index] = new
    picked.append(index)
  picked.sort()
  la, lb = len(tokens_a), len(tokens_b)
  return out[1:1 + la], out[2 + la:2 + la + lb], picked, [tokens[i] for i in picked]


def bert_pairs(docs, di, max_seq_length, short_seq_prob, rnd, masking=None):
  """One document -> list of pairs (a_sents, b_sents, a_win, b_win, is_random_next[, mask]).

  a_sents/b_sents: list of (doc, sentence) ids; *_win: [lo, hi) over their
  concatenated tokens.  masking = (ratio, n_vocab, cls_id, sep_id, mask_id)
  appends mask = (A', B', positions, labels) from masked_lm."""
  document = docs[di]
  max_num_tokens = max_seq_length - 3
  target = max_num_tokens
  if rnd.random() < short_seq_prob:
    target = rnd.randint(2, max_num_tokens)
  out = []
  chunk = []
  cur = 0
  i = 0
  while i < len(document):
    chunk.append(i)
    cur += len(document[i])
    if i == len(document) - 1 or cur >= target:
      if chunk:
        a_end = 1
        if len(chunk) >= 2:
          a_end = rnd.randint(1, len(chunk) - 1)
        a_s = [(di, chunk[j]) for j in range(a_end)]
        la = sum(len(document[chunk[j]]) for j in range(a_end))
        b_s = []
        if len(chunk) == 1 or rnd.random() < 0.5:
          is_random_next = True
          target_b = target - la
          for _ in range(10):
            rdi = rnd.randint(0, len(docs) - 1)
            if rdi != di:
              break
          if rdi == di:
            is_random_next = False
          rdoc = docs[rdi]
          rstart = rnd.randint(0, len(rdoc) - 1)
          lb = 0
          for j in range(rstart, len(rdoc)):
            b_s.append((rdi, j))
            lb += len(rdoc[j])
            if lb >= target_b:
              break
          i -= len(chunk) - a_end
        else:
          is_random_next = False
          b_s = [(di, chunk[j]) for j in range(a_end, len(chunk))]
          lb = sum(len(document[chunk[j]]) for j in range(a_end, len(chunk)))
        a_w, b_w = [0, la], [0, lb]
        _truncate_seq_pair(a_w, b_w, max_num_tokens, rnd)
        assert a_w[1] - a_w[0] >= 1 and b_w[1] - b_w[0] >= 1
        if masking is not None:
          ta = [t for (d, s) in a_s for t in docs[d][s]][a_w[0]:a_w[1]]
          tb = [t for (d, s) in b_s for t in docs[d][s]][b_w[0]:b_w[1]]
          out.append((a_s, b_s, a_w, b_w, is_random_next, masked_lm(ta, tb, *masking, rnd)))
        else:
          out.append((a_s, b_s, a_w, b_w, is_random_next))
      chunk = []
      cur = 0
    i += 1
  return out


def _truncate_seq(w, max_num_tokens, rnd):
  # pretrain_codebert.py:236-247; IndexError when asked to delete from empty
  while True:
    if w[1] - w[0] <= max_num_tokens:
      break
    if w[1] - w[0] == 0:
      raise IndexError('pop from empty list')
    if rnd.random() < 0.5:
      w[0] += 1
    else:
      w[1] -= 1


def codebert_pairs(docs, doc_nseg, di, max_seq_length, short_seq_prob, rnd):
  """docs[di] = list of segments: the first doc_nseg[di] are docstring
  segments, the rest code segments.  Returns list of
  (doc_s, code_s, doc_win, code_win)."""
  segs = docs[di]
  nd = doc_nseg[di]
  dsegs = segs[:nd]
  csegs = segs[nd:]
  special = 3 if nd else 2
  max_num_tokens = max_seq_length - special
  max_doc = 64 if max_seq_length >= 512 else 32
  target = max_num_tokens
  p = rnd.random()
  doc_s = []
  if nd and p < short_seq_prob:
    doc_s = [(di, 0)]
    doc_w = [0, len(dsegs[0])]
  else:
    doc_w = [0, 0]
    chunk = []
    cur = 0
    i = 0
    while i < nd:
      chunk.append(i)
      cur += len(dsegs[i])
      # quirk kept: compares with the CODE segment count (pretrain_codebert.py:382)
      if i == len(csegs) - 1 or cur > max_doc:
        if chunk:
          end = len(chunk) - 1 if (cur > max_doc and len(chunk) > 1) else len(chunk)
          doc_s = [(di, chunk[j]) for j in range(end)]
          doc_w = [0, sum(len(dsegs[chunk[j]]) for j in range(end))]
          _truncate_seq(doc_w, max_doc, rnd)
          break
      i += 1
  doc_len = doc_w[1] - doc_w[0]
  out = []
  chunk = []
  cur = doc_len
  i = 0
  while i < len(csegs):
    chunk.append(i)
    cur += len(csegs[i])
    if i == len(csegs) - 1 or cur > target:
      stay = []
      if chunk:
        if cur > max_num_tokens and len(chunk) > 1:
          stay = [chunk[-1]]
        code_s = [(di, nd + j) for j in chunk]
        code_w = [0, sum(len(csegs[j]) for j in chunk)]
        _truncate_seq(code_w, max_num_tokens - doc_len, rnd)
        assert code_w[1] - code_w[0] >= 1
        if not out or code_w[1] - code_w[0] >= 16:
          out.append((list(doc_s), code_s, list(doc_w), code_w))
      chunk = stay
      cur = sum(len(csegs[j]) for j in chunk) + doc_len
    i += 1
  return out


def partition_pairs(docs, seed, fn, dup):
  """_to_partition_pairs: dup passes, then one shuffle (same RNG stream)."""
  rnd = random.Random(seed)
  pairs = []
  for _ in range(dup):
    for di in range(len(docs)):
      pairs.extend(fn(docs, di, rnd))
  rnd.shuffle(pairs)
  return pairs


def bin_of(num_tokens, bin_size, nbins):
  b = (num_tokens - 1) // bin_size
  return nbins - 1 if b > nbins - 1 else b


def binned_order(num_tokens, bin_size, nbins):
  """stable grouping by bin (binning.py:70-75): list of indices, counts"""
  bins = [[] for _ in range(nbins)]
  for i, n in enumerate(num_tokens):
    bins[bin_of(n, bin_size, nbins)].append(i)
  return [i for b in bins for i in b], [len(b) for b in bins]


# ---------------------------------------------------------------------------
# helpers: corpus arrays -> documents, pairs -> token rows


def filtered_docs(ids, ntok, sent_off, doc_sent_off, d0, d1):
  """Token-id documents of docs [d0, d1) with empty sentences/docs dropped."""
  base = sent_off[0]
  docs = []
  for d in range(d0, d1):
    sents = []
    for s in range(doc_sent_off[d], doc_sent_off[d + 1]):
      n = int(ntok[s])
      if n > 0:
        o = int(sent_off[s] - base)
        sents.append([int(x) for x in ids[o:o + n]])
    if sents:
      docs.append(sents)
  return docs


def pair_tokens(docs, pair):
  a_s, b_s, a_w, b_w, rn = pair[:5]
  a = [t for (d, s) in a_s for t in docs[d][s]][a_w[0]:a_w[1]]
  b = [t for (d, s) in b_s for t in docs[d][s]][b_w[0]:b_w[1]]
  return a, b, rn


def run_bert_shards(corpus, ids, ntok, part_doc_off, target_seq_length, short_seq_prob, dup, seed,
                    bin_size=None, masking=None):
  """Every partition of a corpus -> list (per partition) of rows
  (A ids, B ids, is_random_next, num_tokens[, positions, labels]), in the
  reference's output order (binned when bin_size is given); with masking
  (see bert_pairs) A/B are the masked segments."""
  out = []
  for p in range(len(part_doc_off) - 1):
    docs = filtered_docs(ids, ntok, corpus.sent_off, corpus.doc_sent_off,
                         int(part_doc_off[p]), int(part_doc_off[p + 1]))
    pairs = partition_pairs(docs, seed + p,
                            lambda D, di, r: bert_pairs(D, di, target_seq_length, short_seq_prob, r, masking),
                            dup)
    rows = []
    for pr in pairs:
      a, b, rn = pair_tokens(docs, pr)
      if masking is not None:
        ma, mb, pos, lab = pr[5]
        rows.append((ma, mb, rn, len(a) + len(b) + 3, pos, lab))
      else:
        rows.append((a, b, rn, len(a) + len(b) + 3))
    if bin_size is not None:
      nbins = target_seq_length // bin_size
      order, _ = binned_order([r[3] for r in rows], bin_size, nbins)
      rows = [rows[i] for i in order]
    out.append(rows)
  return out
