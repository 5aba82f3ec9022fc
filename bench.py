#!/usr/bin/env python3
"""Benchmark of the hot path (tokenize -> NSP pack -> bin -> materialise).

Workload (BASELINE.json configs[1]): BERT, --target-seq-length 512,
--bin-size 64, --duplicate-factor 5, bert-base-uncased vocab, a 20 GB
synthetic Wikipedia-style sentence-split corpus resident in HBM per GPU.  One
step = one pass of the whole hot path over that corpus.  Multi-GPU: one
process per GPU (torch.distributed.run), every rank packs its own 20 GB of
partitions (weak scaling, no data-path collective); the per-(partition, bin)
row counts are all-gathered over RCCL at the end of each step (the exchange
that replaces load_balance.py:222-233's MPI Allreduce).

Synthetic data: a unique corpus of --unique-mb MB is generated on the host
and tiled on the device up to --corpus-gb (every tile is its own set of
partitions with its own seeds).  See DESIGN.md "Measurement".

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = 'WordPiece tokens/sec (node) BERT seq128/512 at 1-8 GPUs; % HBM roofline'
HBM_PEAK_GBS = 8000.0


def parse():
  ap = argparse.ArgumentParser()
  ap.add_argument('--gpus', type=int, default=None, help='ranks (default: WORLD_SIZE, else 1)')
  ap.add_argument('--steps', type=int, default=3)
  ap.add_argument('--warmup', type=int, default=1)
  ap.add_argument('--corpus-gb', type=float, default=20.0)
  ap.add_argument('--corpus', choices=('wiki', 'code', 'wikibooks'), default='wiki',
                  help='wiki: BERT on Wikipedia-style text (configs[1]); code: CodeBERT codebert_52000 vocab on '
                       'code-style CodeSearchNet lines (configs[2], one GPU of it); wikibooks: Wikipedia + '
                       'Books-style text (configs[4]: 200 GB over 8 GPUs = --corpus-gb 25 per GPU)')
  ap.add_argument('--unique-mb', type=int, default=None, help='unique synthetic MB (default 256 wiki / 16 code)')
  ap.add_argument('--target-seq-length', type=int, default=512)
  ap.add_argument('--bin-size', type=int, default=64)
  ap.add_argument('--duplicate-factor', type=int, default=None,
                  help='default 5 for BERT (pretrain.py:693), 1 for CodeBERT (pretrain_codebert.py:725)')
  ap.add_argument('--partition-mb', type=float, default=1.0, help='bytes per partition (--block-size)')
  ap.add_argument('--seed', type=int, default=12345)
  ap.add_argument('--masking', action='store_true', help='static masking (--masking of the reference)')
  ap.add_argument('--rows', choices=('spans', 'materialize'), default='spans',
                  help='the step\'s row output: spans of the dense ids (lddl_row_spans, what the writer renders '
                       'from; with --masking + lddl_masked_lm_spans) or materialised token rows (lddl_materialize '
                       '[+ lddl_masked_lm])')
  ap.add_argument('--no-cpu-baseline', action='store_true')
  ap.add_argument('--no-sample-check', action='store_true',
                  help='skip the oracle comparison of one full-size partition after the timed steps')
  ap.add_argument('--cpu-seconds', type=float, default=12.0)
  ap.add_argument('--frontend-mb', type=float, default=100.0,
                  help='MB of raw input for the front-end leg (the preprocessor CLI end to end on BASELINE '
                       'configs[0]: seq 128, no binning; rank 0 at N=1, before the bench touches the GPU; 0: off)')
  ap.add_argument('--parquet-parts', type=int, default=256,
                  help='after timing: write this many partitions as parquet shards and report the writer rate '
                       '(GPU string rendering + host Arrow/parquet encode; 0 = skip)')
  ap.add_argument('--legs', default='mask512,mask128,code,wikibooks',
                  help='after the headline (rank 0 at N=1, outside its timed region): the other BASELINE workloads '
                       'as short legs, each with its own steps, kernel times and oracle check of one full-size '
                       'partition -- mask512 / mask128: static masking at seq 512 / 128 over the same corpus '
                       '(configs[3]), code: CodeBERT seq 512 (configs[2]), wikibooks: Wikipedia + Books seq 512 '
                       '(configs[4]); comma list, "" or none = none')
  ap.add_argument('--leg-steps', type=int, default=2)
  # (measured slower: 124.6 vs 122.0 ms per step, profiles/r6/ov1_*; not the default)
  ap.add_argument('--overlap', dest='overlap', action='store_true', default=False,
                  help='step k pack beside step k+1 tokenize on two streams (unmasked)')
  ap.add_argument('--no-overlap', dest='overlap', action='store_false')
  ap.add_argument('--overlap-priority', type=int, default=1,
                  help='with --overlap: the pack stream at the higher stream priority (1) or the same (0)')
  ap.add_argument('--frontend-c2-mb', type=float, default=2048.0,
                  help='MB of raw input for the C2-scale CLI leg (seq 512, bin 64: BASELINE configs[1] end to '
                       'end through the preprocessor CLI, rank 0 at N=1, before the GPU is touched; 0: off)')
  ap.add_argument('--launch-check', action='store_true',
                  help='multi-rank plumbing only (CPU, gloo, no GPU kernels): launch --gpus ranks, all-gather '
                       'synthetic per-(partition, bin) counts and print the line fields that depend on the world')
  ap.add_argument('--build-check', action='store_true',
                  help='with --launch-check: every rank also runs the library build (a no-op after the launching '
                       'process built it), loads the library and reports its SHA-1')
  args = ap.parse_args()
  code = args.corpus == 'code'
  if args.unique_mb is None:
    args.unique_mb = 16 if code else 256
  if args.duplicate_factor is None:
    args.duplicate_factor = 1 if code else 5
  return args


def build_shards(args, rank, device):
  from lddl_amd import synth
  from lddl_amd.pipeline import ShardSet, partition_by_bytes
  t0 = time.time()
  if args.corpus == 'code':
    # ~1.7 KB per CodeSearchNet-style line (docstring + code segments)
    base = synth.make_code(max(1, (args.unique_mb << 20) // 1700), seed=20261015 + rank)
  elif args.corpus == 'wikibooks':
    base = synth.make_wikibooks(args.unique_mb << 20, seed=20261015 + rank)
  else:
    base = synth.make_wiki(args.unique_mb << 20, seed=20261015 + rank)
  gen_s = time.time() - t0
  nb = base.nbytes
  reps = max(1, int(round(args.corpus_gb * (1 << 30) / nb)))
  n_part_base = max(1, int(round(nb / (args.partition_mb * (1 << 20)))))
  pdo = partition_by_bytes(base, n_part_base)
  ns, nd, npb = base.n_sent, base.n_doc, len(pdo) - 1
  data = torch.empty(nb * reps + 16, dtype=torch.uint8, device=device)
  src = torch.from_numpy(base.data[:nb]).to(device)
  for r in range(reps):
    data[r * nb:(r + 1) * nb].copy_(src)
  data[nb * reps:].zero_()
  del src
  so = torch.from_numpy(base.sent_off - base.sent_off[0]).to(device)
  sent_off = torch.empty(ns * reps + 1, dtype=torch.int64, device=device)
  dso = torch.from_numpy(base.doc_sent_off).to(device)
  doc_sent_off = torch.empty(nd * reps + 1, dtype=torch.int64, device=device)
  pd = torch.from_numpy(pdo).to(device)
  part_doc_off = torch.empty(npb * reps + 1, dtype=torch.int64, device=device)
  nseg = None
  if base.doc_nseg_doc is not None:
    nseg = torch.from_numpy(np.tile(base.doc_nseg_doc, reps)).to(device)
  for r in range(reps):
    sent_off[r * ns:(r + 1) * ns + 1] = so + r * nb
    doc_sent_off[r * nd:(r + 1) * nd + 1] = dso + r * ns
    part_doc_off[r * npb:(r + 1) * npb + 1] = pd + r * nd
  sh = ShardSet(data, sent_off, doc_sent_off, part_doc_off, nseg, nb * reps)
  return sh, base, pdo, reps, gen_s


def _code_docs(base, ids, ntok, d0, d1):
  """CodeBERT documents of docs [d0, d1): (docstring + code segments, #docstring
  segments), empty segments dropped, docs without code dropped
  (pretrain_codebert.py:126-161)"""
  docs, nd = [], []
  for d in range(d0, d1):
    ss = [list(map(int, ids[base.sent_off[s] - base.sent_off[0]:base.sent_off[s] - base.sent_off[0] + ntok[s]]))
          for s in range(base.doc_sent_off[d], base.doc_sent_off[d + 1])]
    k = int(base.doc_nseg_doc[d])
    ds = [s for s in ss[:k] if s]
    cs = [s for s in ss[k:] if s]
    if cs:
      docs.append(ds + cs)
      nd.append(len(ds))
  return docs, nd


def _ref_tok_worker(a):
  """one host process: the reference's per-sentence tokenize call over its
  sentences for ~seconds -> (tokens, sentences, elapsed)"""
  vocab, sents, seconds = a
  import transformers
  tok = transformers.BertTokenizerFast(vocab)
  n = k = 0
  t = time.perf_counter()
  while k < len(sents) and (k & 255 or time.perf_counter() - t < seconds):
    n += min(512, len(tok.tokenize(sents[k], max_length=512, truncation=True)))
    k += 1
  return n, k, time.perf_counter() - t


def reference_tokenizer_rate(args, base, seconds, procs):
  """The reference's own tokenizer call (pretrain.py:79-80: HF
  BertTokenizerFast(vocab).tokenize(s, max_length=512, truncation=True), one
  Python call per sentence in each single-threaded Dask worker), run by
  `procs` host processes at once (the reference runs one such worker per
  core), each over its own sentences of the same corpus for ~seconds; the
  node rate is the sum of the per-process rates.  None when transformers is
  not importable."""
  try:
    import transformers
  except Exception:
    return None
  import multiprocessing
  from lddl_amd.pipeline import VOCAB_BERT, VOCAB_CODEBERT
  vocab = VOCAB_CODEBERT if args.corpus == 'code' else VOCAB_BERT
  per = min(base.n_sent // max(1, procs), 30_000)
  work = [(vocab, [base.sentence(k) for k in range(i * per, (i + 1) * per)], seconds) for i in range(procs)]
  # spawned (not forked) workers: this process holds a GPU context
  with multiprocessing.get_context('spawn').Pool(procs) as pool:
    out = pool.map(_ref_tok_worker, work)
  rates = [n / el for n, k, el in out]
  return {'value': sum(rates), 'tokens_per_s_per_core': float(np.mean(rates)), 'unit': 'tokens/s', 'cores': procs,
          'kind': 'reference-library',
          'sample': 'transformers %s BertTokenizerFast.tokenize per sentence (the call at pretrain.py:79-80) in %d '
                    'host processes at once, %d sentences in %.1f s each on average' % (
                        transformers.__version__, procs, int(np.mean([k for n, k, el in out])),
                        float(np.mean([el for n, k, el in out])))}


def cpu_baseline(args, base, pdo, seconds):
  """oracle/ restatement timed on the host cores on a bounded sample."""
  from oracle.oracle import OracleTokenizer
  from oracle import pack_oracle as po
  from lddl_amd.pipeline import VOCAB_BERT, VOCAB_CODEBERT
  code = args.corpus == 'code'
  hc = host_cpus()
  threads = hc['share']
  ot = OracleTokenizer(VOCAB_CODEBERT if code else VOCAB_BERT)
  # calibrate on ~1 MB, then size the sample to ~seconds of work
  ns = int(np.searchsorted(base.sent_off, base.sent_off[0] + (1 << 20)))
  # output buffers allocated and touched outside the timed calls (page faults
  # of a fresh 4-B-per-byte array otherwise serialise the threads)
  out = (np.zeros(base.nbytes + 16, np.int32), np.zeros(base.n_sent + 1, np.int32))
  out[0].fill(1)
  out[1].fill(1)
  t = time.time()
  ot.run(base.data, base.sent_off[:ns + 1], 512, nthreads=threads, out=out)
  rate = (base.sent_off[ns] - base.sent_off[0]) / max(1e-6, time.time() - t)
  # one thread on ~1 s of the same text: the per-core rate and how the
  # tokenizer scales from 1 to `threads` cores (the box projection's basis)
  n1 = int(np.searchsorted(base.sent_off, base.sent_off[0] + int(rate / max(1, threads))))
  n1 = max(1, min(n1, base.n_sent))
  t = time.time()
  ot.run(base.data, base.sent_off[:n1 + 1], 512, nthreads=1, out=out)
  rate1 = float(out[1][:n1].sum()) / max(1e-6, time.time() - t)
  want = min(base.nbytes, int(rate * seconds * 0.7))
  ns = int(np.searchsorted(base.sent_off, base.sent_off[0] + want))
  ns = max(1, min(ns, base.n_sent))
  t = time.time()
  ids, ntok = ot.run(base.data, base.sent_off[:ns + 1], 512, nthreads=threads, out=out)
  tok_s = time.time() - t
  ntok = ntok[:ns]
  tok_rate = float(ntok.sum()) / tok_s
  # pack+bin (pure-Python restatement, 1 thread) on the first partitions
  t = time.time()
  ptoks, p = 0, 0
  while time.time() - t < seconds * 0.3 and p < len(pdo) - 1 and base.doc_sent_off[pdo[p + 1]] <= ns:
    if code:
      docs, nd = _code_docs(base, ids, ntok, int(pdo[p]), int(pdo[p + 1]))
      pairs = po.partition_pairs(docs, args.seed + p, lambda D, di, r: po.codebert_pairs(
          D, nd, di, args.target_seq_length, 0.1, r), args.duplicate_factor)
      nt = []
      for (doc_s, code_s, dw, cw) in pairs:
        dt = [t for (d, s) in doc_s for t in docs[d][s]][dw[0]:dw[1]]
        ct = [t for (d, s) in code_s for t in docs[d][s]][cw[0]:cw[1]]
        nt.append(len(dt) + len(ct) + (3 if nd[code_s[0][0]] else 2))
    else:
      docs = po.filtered_docs(ids, ntok, base.sent_off, base.doc_sent_off, int(pdo[p]), int(pdo[p + 1]))
      pairs = po.partition_pairs(docs, args.seed + p, lambda D, di, r: po.bert_pairs(
          D, di, args.target_seq_length, 0.1, r), args.duplicate_factor)
      rows = [po.pair_tokens(docs, pr) for pr in pairs]
      nt = [len(a) + len(b) + 3 for a, b, _ in rows]
    po.binned_order(nt, args.bin_size, args.target_seq_length // args.bin_size)
    ptoks += int(sum(ntok[base.doc_sent_off[pdo[p]]:base.doc_sent_off[pdo[p + 1]]]))
    p += 1
  pack_s = time.time() - t
  pack_rate = ptoks / pack_s if p else None
  # end-to-end CPU rate: tokenize at `threads`, pack at 1 thread x `threads` processes
  e2e = None
  if pack_rate:
    e2e = 1.0 / (1.0 / tok_rate + 1.0 / (pack_rate * threads))
  ref = reference_tokenizer_rate(args, base, min(3.0, seconds * 0.25), threads)
  eff = tok_rate / (threads * rate1) if rate1 > 0 else None
  box = hc['affinity'] or threads
  proj = None
  if box > threads and eff:
    # NOT measured: this harness caps a GPU command's worker pools at the box's
    # CPU share (16 per GPU); the whole box's rate is the measured rate at
    # `threads` cores scaled linearly to the affinity count
    proj = {'cores': box, 'tokenize_tokens_per_s': tok_rate * box / threads,
            'value': (e2e if e2e else tok_rate) * box / threads,
            'basis': 'measured at %d cores (%.2f of linear from 1 core), scaled linearly to the %d-CPU affinity; '
                     'not measured (worker pools are capped at the box CPU share)' % (threads, eff, box)}
  return {'value': e2e if e2e else tok_rate, 'unit': 'tokens/s', 'cores': threads, 'kind': 'port',
          'tokenize_scaling_1_to_%d' % threads: eff, 'tokenize_tokens_per_s_1_core': rate1,
          'projected_box': proj,
          'reference_library': ref,
          'sample': ('oracle/tokenizer_oracle.c on %d sentences (%.1f MB, %.1f s, %.3g tok/s at %d threads) + '
                     'oracle/pack_oracle.py on %d partitions (%.1f s, %.3g input tok/s/thread); value = '
                     'tokenize and pack at %d cores in series' % (
                         ns, (base.sent_off[ns] - base.sent_off[0]) / 1e6, tok_s, tok_rate, threads, p, pack_s,
                         pack_rate or 0, threads)),
          'tokenize_tokens_per_s': tok_rate, 'pack_tokens_per_s_per_thread': pack_rate,
          'host_cpus': hc}


def host_cpus():
  """The box's CPU count, this process's affinity, the cgroup quota and the
  share the CPU legs run at (lddl_amd.hostinfo): min(affinity, LDDL_CPU_SHARE
  or 16).  The GPU boxes of this harness show the whole machine in
  os.cpu_count() / the affinity (256) and allot one GPU's command a share of
  16 cores for its worker pools -- the box exports OMP_NUM_THREADS / MAX_JOBS
  = 16 to say so, and `evidence` carries those variables and the cgroup's
  cpu.max as the box shows them."""
  from lddl_amd import hostinfo
  ev = hostinfo.cpu_evidence()
  return {'os_cpu_count': ev['os_cpu_count'], 'affinity': ev['affinity'], 'share': hostinfo.cpu_share(),
          'evidence': ev}


def sample_partition_check(args, pk, res, base, pdo, reps, seed0):
  """One full-size partition of the timed run (the middle partition of the
  middle replica) against the oracle, outside the timed region: its rows
  (partition, A, B, is_random_next, num_tokens[, masked positions / labels])
  in output order must be identical."""
  from oracle.oracle import OracleTokenizer
  from oracle import pack_oracle as po
  from lddl_amd.synth import Corpus
  t0 = time.time()
  code = args.corpus == 'code'
  npb = len(pdo) - 1
  r, q = reps // 2, npb // 2
  p = r * npb + q
  bc = res.bin_count.cpu().numpy()
  g0, n = int(bc[:p].sum()), int(bc[p].sum())
  off = res.tok_off[g0:g0 + n + 1].cpu().numpy()
  l0 = res.len0[g0:g0 + n].cpu().numpy().view(np.uint16).astype(np.int64)
  l1 = res.len1[g0:g0 + n].cpu().numpy().view(np.uint16).astype(np.int64)
  fl = res.flags[g0:g0 + n].cpu().numpy()
  if res.spans:  # the rows rebuilt from the spans over the dense ids
    s0 = res.src0[g0:g0 + n].cpu().numpy()
    s1 = res.src1[g0:g0 + n].cpu().numpy()
    lo, hi = int(min(s0.min(), s1.min())), int(max((s0 + l0).max(), (s1 + l1).max()))
    ids = res.ids[lo:hi].cpu().numpy().view(np.uint16).astype(np.int64)
    rws = [np.concatenate([[res.cls_id], ids[s0[g] - lo:s0[g] - lo + l0[g]], [res.sep_id] if fl[g] & 2 else [],
                           ids[s1[g] - lo:s1[g] - lo + l1[g]], [res.sep_id]]).astype(np.int64) for g in range(n)]
    if res.mlm_token is not None:  # the masked rows show mlm_token at mlm_pos
      mo = res.mlm_off[g0:g0 + n + 1].cpu().numpy()
      mp = res.mlm_pos[int(mo[0]):int(mo[-1])].cpu().numpy().view(np.uint16).astype(np.int64)
      mt = res.mlm_token[int(mo[0]):int(mo[-1])].cpu().numpy().view(np.uint16).astype(np.int64)
      for g in range(n):
        rws[g][mp[mo[g] - mo[0]:mo[g + 1] - mo[0]]] = mt[mo[g] - mo[0]:mo[g + 1] - mo[0]]
    tok = np.concatenate(rws)
  else:
    tok = res.tokens[int(off[0]):int(off[-1])].cpu().numpy().view(np.uint16).astype(np.int64)
  pt = res.part[g0:g0 + n].cpu().numpy()
  if res.mlm_off is not None:
    moff = res.mlm_off[g0:g0 + n + 1].cpu().numpy()
    mpos = res.mlm_pos[int(moff[0]):int(moff[-1])].cpu().numpy().view(np.uint16).astype(np.int64)
    mlab = res.mlm_label[int(moff[0]):int(moff[-1])].cpu().numpy().view(np.uint16).astype(np.int64)
  got = []
  for g in range(n):
    row = tok[off[g] - off[0]:off[g + 1] - off[0]]
    k0 = 1 + int(l0[g]) + (1 if fl[g] & 2 else 0)
    e = (int(pt[g]), row[1:1 + l0[g]].tolist(), row[k0:k0 + l1[g]].tolist(), int(fl[g]) & 1, len(row))
    if res.mlm_off is not None:
      e += (mpos[moff[g] - moff[0]:moff[g + 1] - moff[0]].tolist(), mlab[moff[g] - moff[0]:moff[g + 1] - moff[0]].tolist())
    got.append(e)
  # the oracle over the partition's documents of the unique corpus
  d0, d1 = int(pdo[q]), int(pdo[q + 1])
  s0, s1 = int(base.doc_sent_off[d0]), int(base.doc_sent_off[d1])
  b0 = int(base.sent_off[s0])
  sub = Corpus(np.ascontiguousarray(base.data[b0:int(base.sent_off[s1])]), base.sent_off[s0:s1 + 1] - b0,
               base.doc_sent_off[d0:d1 + 1] - s0,
               None if base.doc_nseg_doc is None else base.doc_nseg_doc[d0:d1])
  oids, ontok = OracleTokenizer(pk.tok.vocab_file).run(sub.data, sub.sent_off, 512,
                                                        nthreads=host_cpus()['share'])
  nbins = args.target_seq_length // args.bin_size
  if code:
    docs, nd = _code_docs(sub, oids, ontok, 0, d1 - d0)
    pairs = po.partition_pairs(docs, seed0 + p, lambda D, di, rr: po.codebert_pairs(
        D, nd, di, args.target_seq_length, 0.1, rr), args.duplicate_factor)
    rows = []
    for (doc_s, code_s, dw, cw) in pairs:
      dt = [t for (d, x) in doc_s for t in docs[d][x]][dw[0]:dw[1]]
      ct = [t for (d, x) in code_s for t in docs[d][x]][cw[0]:cw[1]]
      rows.append((dt, ct, 0, len(dt) + len(ct) + (3 if nd[code_s[0][0]] else 2)))
    order, _ = po.binned_order([x[3] for x in rows], args.bin_size, nbins)
    exp = [rows[i] for i in order]
  else:
    mask = (0.15, pk.tok.vocab_size, pk.tok.cls_id, pk.tok.sep_id, pk.tok.mask_id) if args.masking else None
    exp = po.run_bert_shards(sub, oids, ontok, [0, d1 - d0], args.target_seq_length, 0.1, args.duplicate_factor,
                             seed0 + p, args.bin_size, mask)[0]
  exp = [(p, list(x[0]), list(x[1]), int(bool(x[2])), x[3]) + ((list(x[4]), list(x[5])) if len(x) > 4 else ())
         for x in exp]
  if code:  # (CodeBERT rows carry no is_random_next)
    got = [(x[0], x[1], x[2], 0) + x[4:] for x in got]
  if got != exp:
    bad = next(i for i, (a, b) in enumerate(zip(got + [None] * len(exp), exp + [None] * len(got))) if a != b)
    raise RuntimeError('sampled partition %d differs from the oracle at row %d of %d / %d' % (p, bad, len(got),
                                                                                            len(exp)))
  return {'partition': p, 'rows': n, 'sentences': s1 - s0, 'identical': True, 'seconds': time.time() - t0}


def parquet_sample(args, pk, res, sh, enc=None):
  """Writer throughput on the first --parquet-parts partitions (outside the
  timed step; the reference's to_parquet_binned stage, reported separately).
  enc: the process encoder (writer.ProcessEncoder, started before the GPU),
  else the writer's thread pool"""
  import shutil
  import tempfile
  from lddl_amd import writer
  d = tempfile.mkdtemp(prefix='lddl_bench_pq_')
  doc_ids = None
  if args.corpus == 'code':  # the CodeBERT 'id' column of the documents written
    nd = int(sh.part_doc_off[min(args.parquet_parts, sh.n_part)].item())
    import pyarrow as pa  # (as the CLI's split workers hand it over: an Arrow column)
    doc_ids = pa.array(['python_%d' % i for i in range(nd)], type=pa.string())
  try:
    # one untimed partition first: pyarrow's lazily imported modules (compute,
    # pandas compat: ~0.55 s once per process) stay out of the rate
    pend = []
    writer.write_shards(pk, res, os.path.join(d, 'warm'), bin_size=args.bin_size, masking=args.masking,
                        codebert=args.corpus == 'code', doc_ids=doc_ids, max_parts=1, executor=enc, pending=pend)
    for f_ in pend:
      f_.result()
    pend = []
    torch.cuda.synchronize()
    t = time.perf_counter()
    files = writer.write_shards(pk, res, d, bin_size=args.bin_size, masking=args.masking,
                                codebert=args.corpus == 'code', doc_ids=doc_ids,
                                max_parts=args.parquet_parts, executor=enc, pending=pend)
    for f_ in pend:
      f_.result()
    el = time.perf_counter() - t
    nbytes = sum(os.path.getsize(f) for f in files)
    nb = res.nbins
    rows = int(res.bin_count[:args.parquet_parts].sum().item())
    return {'partitions': args.parquet_parts, 'files': len(files), 'rows': rows, 'seconds': el,
            'rows_per_s': rows / el, 'parquet_mb': nbytes / 1e6, 'compression': 'snappy', 'nbins': nb,
            'sink': d, 'encoder': 'processes' if enc is not None else 'threads', 'stages': dict(writer.LAST_STATS)}
  finally:
    shutil.rmtree(d, ignore_errors=True)


def frontend_leg(mb, chunk_mb=32.0, seq=128, bin_size=None, unique_mb=256):
  """The preprocessor CLI end to end (lddl_amd.preprocess.main, the
  reference's preprocess_bert_pretrain) on mb MB of synthetic Wikipedia-style
  raw input (one ``wiki-<id> <text>`` document per line): BASELINE.json
  configs[0] (seq 128, no static masking, unbinned parquet) by default,
  configs[1] with seq=512, bin_size=64.  Past unique_mb the documents repeat
  (each line keeps its own id).  Runs in a child process of its own, as the
  command line does, started before this process touches the GPU; wall,
  host read / sentence split / GPU / parquet write seconds and the split
  time hidden behind the GPU and the writer, as preprocess.main reports
  them (main() itself: interpreter start-up and imports excluded), and the
  CPU seconds of the CLI process and of its reaped workers (split pool,
  encoders) over the run: against host_cpus share x wall, whether the leg
  is CPU-bound."""
  import shutil
  import tempfile
  from lddl_amd import synth
  d = tempfile.mkdtemp(prefix='lddl_bench_fe_')
  try:
    t0 = time.perf_counter()
    c = synth.make_wiki(int(min(mb, unique_mb) * (1 << 20)), seed=11)
    data, so, dso = c.data.tobytes(), c.sent_off, c.doc_sent_off
    lines = [b' '.join(data[so[k]:so[k + 1]] for k in range(dso[q], dso[q + 1])) for q in range(c.n_doc)]
    os.makedirs(os.path.join(d, 'wiki', 'en'))
    want, i = int(mb * (1 << 20)), 0
    with open(os.path.join(d, 'wiki', 'en', 'a.txt'), 'wb') as f:
      while f.tell() < want:
        for doc in lines:
          f.write(b'wiki-%d %s\n' % (i, doc))
          i += 1
    gen_s = time.perf_counter() - t0
    raw = os.path.getsize(os.path.join(d, 'wiki', 'en', 'a.txt'))
    argv = ['--wikipedia', os.path.join(d, 'wiki'), '--sentence-splitter', 'rules', '--sink', os.path.join(d, 'out'),
            '--target-seq-length', str(seq), '--block-size', '1M', '--chunk-mb', str(chunk_mb), '--seed', '7',
            '--split-workers', str(host_cpus()['share'])]
    if bin_size:
      argv += ['--bin-size', str(bin_size)]
    # a child process per CLI run, as the command line runs it: its GPU
    # context, split pool and encoders start and end with it (run in this
    # process, the second leg paid the first leg's context teardown); the
    # module imports (torch, ~1.5 s cold) are timed on their own: imports_s
    code = ('import json, sys, time; t0 = time.perf_counter(); import torch; '
            'from lddl_amd import preprocess, pipeline, writer, balance; imp = time.perf_counter() - t0; '
            'a = preprocess.attach_args().parse_args(json.loads(sys.argv[1])); '
            'import resource; r0 = resource.getrusage(resource.RUSAGE_SELF); '
            't0 = time.perf_counter(); files, t = preprocess.main(a); el = time.perf_counter() - t0; '
            'r1 = resource.getrusage(resource.RUSAGE_SELF); rc = resource.getrusage(resource.RUSAGE_CHILDREN); '
            't["cpu_main_s"] = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime); '
            't["cpu_workers_s"] = rc.ru_utime + rc.ru_stime; '
            't.pop("partitions", None); t["files"] = len(files); t["el"] = el; t["imports_s"] = imp; '
            'print("LDDL_LEG " + json.dumps({k: v for k, v in t.items() if isinstance(v, (int, float, str))}))')
    p = subprocess.run([sys.executable, '-c', code, json.dumps(argv)], stdout=subprocess.PIPE,
                       cwd=os.path.dirname(os.path.abspath(__file__)), timeout=900)
    rows = [ln for ln in p.stdout.decode().splitlines() if ln.startswith('LDDL_LEG ')]
    if p.returncode != 0 or not rows:
      raise RuntimeError('preprocess CLI leg failed (exit %d)' % p.returncode)
    t = json.loads(rows[-1][len('LDDL_LEG '):])
    files, el = [None] * t.pop('files'), t.pop('el')
    out = {'what': 'preprocess CLI end to end, BERT seq %d %s (BASELINE configs[%d])' % (
               seq, 'bin %d' % bin_size if bin_size else 'unbinned', 1 if bin_size else 0),
           'raw_mb': raw / 1e6, 'documents': i, 'unique_mb': min(mb, unique_mb),
           'files': len(files), 'seconds': el, 'raw_mb_per_s': raw / 1e6 / el, 'gen_s': gen_s,
           'rows_per_s': t.get('pairs', 0) / el, 'work_dir': tempfile.gettempdir()}
    out.update({k: v for k, v in t.items() if isinstance(v, (int, float, str))})
    return out
  finally:
    shutil.rmtree(d, ignore_errors=True)


def launch_ranks(args):
  """`--gpus N` without a launcher: start N rank processes (this process has
  not touched the GPU: torch.cuda.device_count() does not initialise it) with
  RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* as torch.distributed.run sets them,
  wait for all of them, and return the worst exit code.  Rank 0 prints the
  line."""
  import socket
  import subprocess
  if not args.launch_check:
    have = torch.cuda.device_count()
    if args.gpus > have:
      print('bench.py: --gpus %d but %d GPU(s) visible' % (args.gpus, have), file=sys.stderr)
      return 2
  if not args.launch_check or args.build_check:
    # build once, here, before any rank exists (this process has not touched
    # the GPU): N ranks finding a stale library would otherwise all compile
    # (build_hip's lock serialises them, but each would wait for the first)
    from lddl_amd import build
    build.build_hip()
  with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
  procs = []
  for r in range(args.gpus):
    env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
               MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
  codes = [p.wait() for p in procs]
  bad = [c for c in codes if c != 0]
  return bad[0] if bad else 0


def check_gather(gathered, own, rank, world):
  """the all-gather saw every rank: world x the per-rank partitions, this
  rank's block in its place"""
  n_part = own.shape[0]
  if gathered.shape[0] != world * n_part or not np.array_equal(gathered[rank * n_part:(rank + 1) * n_part], own):
    raise RuntimeError('all-gather of bin counts: %d partitions gathered, expected %d x %d' % (
        gathered.shape[0], world, n_part))
  return int(gathered.shape[0])


def launch_check(args, rank, world):
  """--launch-check: the world-dependent part of a bench run on the CPU (gloo)"""
  import torch.distributed as dist
  from lddl_amd.balance import gather_bin_counts
  if world > 1:
    dist.init_process_group('gloo')
  n_part, nbins = 7, args.target_seq_length // args.bin_size
  own = torch.arange(n_part * nbins, dtype=torch.int64).view(n_part, nbins) + 1000 * rank
  got = gather_bin_counts(own, rank * n_part) if world > 1 else own.numpy()
  n = check_gather(got, own.numpy(), rank, world)
  libs = None
  if args.build_check:  # every rank: build (a no-op now) and load the library it would run
    import ctypes
    import hashlib
    from lddl_amd import build
    path = build.build_hip()
    ctypes.CDLL(path)
    with open(path, 'rb') as f:
      mine = (path, hashlib.sha1(f.read()).hexdigest())
    libs = [None] * world
    if world > 1:
      dist.all_gather_object(libs, mine)
    else:
      libs = [mine]
  if rank == 0:
    print(json.dumps({'metric': METRIC, 'check': 'launch', 'n_gpus': world, 'gathered_partitions': n,
                      'partitions_per_rank': n_part, 'parallelism': 'shard%d' % world, 'libs': libs}), flush=True)
  if world > 1:
    dist.destroy_process_group()


LEGS = {
    'mask512': dict(corpus='wiki', masking=True, target_seq_length=512, bin_size=64, duplicate_factor=5),
    'mask128': dict(corpus='wiki', masking=True, target_seq_length=128, bin_size=64, duplicate_factor=5),
    'code': dict(corpus='code', masking=False, target_seq_length=512, bin_size=64, duplicate_factor=1),
    'wikibooks': dict(corpus='wikibooks', masking=False, target_seq_length=512, bin_size=64, duplicate_factor=5),
}


def run_leg(args, name, local, device, shards=None):
  """One BASELINE workload after the headline (never inside its timed
  region): warmup + --leg-steps timed steps of tokenize + pack (+ masking)
  + bin + row spans at full size, per-kernel tokenizer times of the last
  step, and the oracle check of one full-size partition.  shards: the
  headline's (same corpus) to reuse, else built here."""
  import argparse
  from lddl_amd.pipeline import Packer, VOCAB_BERT, VOCAB_CODEBERT
  a = argparse.Namespace(**vars(args))
  for k, v in LEGS[name].items():
    setattr(a, k, v)
  a.unique_mb = 16 if a.corpus == 'code' else 256
  a.rows = 'spans'
  t0 = time.perf_counter()
  if shards is None:
    sh, base, pdo, reps, _ = build_shards(a, 0, device)
  else:
    sh, base, pdo, reps = shards
  code = a.corpus == 'code'
  pk = Packer(VOCAB_CODEBERT if code else VOCAB_BERT, device=local, masking=a.masking)
  pk.tok.set_timing(True)
  kw = dict(target_seq_length=a.target_seq_length, short_seq_prob=0.1, duplicate_factor=a.duplicate_factor,
       seed=a.seed, bin_size=a.bin_size, masking=a.masking, codebert=code, spans=True)
  ev = []
  for i in range(1 + a.leg_steps):
    if i == 1:
      torch.cuda.synchronize()
      t = time.perf_counter()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    ids, ntok, toff = pk.tokenize(sh)
    e1.record(s)
    res = pk.pack(sh, ids, ntok, toff, **kw)
    if i:
      ev.append((e0, e1))
  torch.cuda.synchronize()
  el = (time.perf_counter() - t) / a.leg_steps
  n_tok = int(ntok[:sh.n_sent].sum().item())
  ks = pk.tok.stats()
  out = {'workload': '%s_seq%d_bin%d_%dGB_per_gpu%s' % ({'code': 'codebert', 'wiki': 'bert',
                             'wikibooks': 'bert_wikibooks'}[a.corpus],
                             a.target_seq_length, a.bin_size,
                             round(sh.nbytes / (1 << 30)),
                             '_masking' if a.masking else ''),
     'baseline_config': {'mask512': 3, 'mask128': 3, 'code': 2, 'wikibooks': 4}[name],
     'steps': a.leg_steps, 'warmup': 1, 'ms_per_step': el * 1e3, 'value': n_tok / el, 'unit': 'tokens/s',
     'duplicate_factor': a.duplicate_factor, 'corpus_bytes': sh.nbytes, 'wordpiece_tokens': n_tok,
     'pairs': res.n_pairs, 'packed_tokens': res.n_tokens, 'masked_positions': res.n_masked,
     'tokenize_ms': float(np.mean([x.elapsed_time(y) for x, y in ev])),
     'tokenize_kernels_ms': {'scan': ks['scan_ms'], 'wordpiece': ks['wordpiece_ms'], 'expand': ks['expand_ms']}}
  try:  # device memory left while the leg's results are live
    out['hbm_free_gb'] = round(torch.cuda.mem_get_info(device)[0] / 1e9, 1)
  except Exception:  # (diagnostic only)
    pass
  if not args.no_sample_check:
    out['sample_check'] = sample_partition_check(a, pk, res, base, pdo, reps, kw['seed'])
  out['leg_seconds'] = time.perf_counter() - t0
  del res, ids, ntok, toff, pk
  return out


_T0 = time.perf_counter()


def progress(rank, msg):
  """a stage mark on stderr (rank 0): long runs show they are alive"""
  if rank == 0:
    print('[bench %7.1fs] %s' % (time.perf_counter() - _T0, msg), file=sys.stderr, flush=True)


def main():
  args = parse()
  if 'WORLD_SIZE' not in os.environ and (args.gpus or 1) > 1:
    sys.exit(launch_ranks(args))
  rank = int(os.environ.get('RANK', 0))
  world = int(os.environ.get('WORLD_SIZE', 1))
  local = int(os.environ.get('LOCAL_RANK', 0))
  if args.gpus is None:
    args.gpus = world
  if world != args.gpus:
    raise SystemExit('bench.py: --gpus %d but WORLD_SIZE=%d' % (args.gpus, world))
  if args.launch_check:
    return launch_check(args, rank, world)
  progress(rank, 'start')
  # the writer sample's encode processes, forked while the process is GPU-free
  # (LDDL_ENCODE_PROCS=0: the thread pool instead)
  enc = None
  if args.parquet_parts > 0 and os.environ.get('LDDL_ENCODE_PROCS', '1') != '0':
    from lddl_amd import writer
    enc = writer.ProcessEncoder()
  def cli_leg(*a, **kw):  # (a failed CLI leg is recorded in the line; the headline still runs)
    try:
      return frontend_leg(*a, **kw)
    except Exception as e:  # noqa: BLE001
      return {'error': '%s: %s' % (type(e).__name__, e)}

  fe = cli_leg(args.frontend_mb) if world == 1 and args.frontend_mb > 0 else None
  progress(rank, 'frontend leg done')
  fe2 = (cli_leg(args.frontend_c2_mb, seq=512, bin_size=64)
         if world == 1 and args.frontend_c2_mb > 0 else None)
  torch.cuda.set_device(local)
  device = torch.device('cuda', local)
  dist = None
  if world > 1:
    import torch.distributed as dist
    dist.init_process_group('nccl', device_id=device)
  from lddl_amd.pipeline import Packer
  from lddl_amd import build
  build.build_hip()
  progress(rank, 'frontend_c2 leg done')
  sh, base, pdo, reps, gen_s = build_shards(args, rank, device)
  progress(rank, 'shards built')
  from lddl_amd.pipeline import VOCAB_BERT, VOCAB_CODEBERT
  code = args.corpus == 'code'
  pk = Packer(VOCAB_CODEBERT if code else VOCAB_BERT, device=local, masking=args.masking)
  pk.tok.set_timing(True)  # per-kernel HIP events inside the tokenize call (the roofline's kernel time)
  kw = dict(target_seq_length=args.target_seq_length, short_seq_prob=0.1, duplicate_factor=args.duplicate_factor,
            seed=args.seed + rank * 10_000_000, bin_size=args.bin_size, masking=args.masking, codebert=code,
            spans=args.rows == 'spans')
  tok_ms = []
  gathered = []

  # Steps overlap pairwise with --overlap (unmasked): step k's pack (scalar-unit
  # bound) runs on its own stream beside step k+1's tokenize (vector-unit and
  # latency bound) on another.  The tokenizer writes alternating output sets
  # (pipeline.TokBuffers), so step k+1's tokenize waits only for the pack
  # of step k-1, the last reader of the set it overwrites.  Every step still
  # tokenizes, packs, bins and writes the row spans of the whole 20 GB; the
  # timed region ends when both streams are idle.
  overlap = args.overlap and not args.masking
  if overlap:
    from lddl_amd.pipeline import TokBuffers
    # (the pack stream at the higher priority: its one-wave blocks dispatch
    # first wherever slots free, and the tokenizer's persistent blocks --
    # which claim their work from counters -- fill what the packer's tail
    # leaves idle)
    lo_pri, hi_pri = torch.cuda.Stream.priority_range()
    st_tok = torch.cuda.Stream(device, priority=lo_pri)
    st_pack = torch.cuda.Stream(device, priority=hi_pri if args.overlap_priority else lo_pri)
    tbufs = [TokBuffers(), TokBuffers()]
    ov = {'k': 0, 'packed': [None, None]}

  def step(timed):
    if overlap:
      i = ov['k'] % 2
      ov['k'] += 1
      s = st_tok
      with torch.cuda.stream(st_tok):
        if ov['packed'][i] is not None:
          st_tok.wait_event(ov['packed'][i])  # (the pack that last read set i)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        ids, ntok, toff = pk.tokenize(sh, stream=st_tok, bufs=tbufs[i])
        e1.record(s)
      with torch.cuda.stream(st_pack):
        st_pack.wait_event(e1)
        res = pk.pack(sh, ids, ntok, toff, stream=st_pack, **kw)
        done = torch.cuda.Event()
        done.record(st_pack)
        ov['packed'][i] = done
    else:
      s = torch.cuda.current_stream()
      e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
      e0.record(s)
      ids, ntok, toff = pk.tokenize(sh)
      e1.record(s)
      res = pk.pack(sh, ids, ntok, toff, **kw)
    if dist is not None:
      # per-(partition, bin) row counts of every rank: the load balancer's
      # input (lddl_amd/balance.py), one RCCL all-gather per step
      from lddl_amd.balance import gather_bin_counts
      with torch.cuda.stream(st_pack if overlap else torch.cuda.current_stream()):
        g = gather_bin_counts(res.bin_count, rank * sh.n_part)
      if timed:
        gathered.append(g)
    if timed:
      tok_ms.append((e0, e1))
    return res, ntok

  for _ in range(args.warmup):
    step(False)
  torch.cuda.synchronize()
  if dist is not None:
    dist.barrier()
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  for _ in range(args.steps):
    res, ntok = step(True)
  torch.cuda.synchronize()
  if dist is not None:
    dist.barrier()
  el = time.perf_counter() - t0
  n_tok = int(ntok[:sh.n_sent].sum().item())
  # full-size property check (outside the timed region): every replica of the
  # unique corpus must tokenize to the same number of tokens
  per_rep = ntok[:reps * base.n_sent].view(reps, base.n_sent).to(torch.int64).sum(1)
  if not bool((per_rep == per_rep[0]).all()):
    raise RuntimeError('tokenize: replicas disagree: %s' % per_rep.tolist()[:16])
  tk = float(np.mean([a.elapsed_time(b) for a, b in tok_ms]))
  ks = pk.tok.stats()  # the last timed step's tokenize kernels
  if not ks['launches'] or ks['scan_ms'] <= 0:
    raise RuntimeError('bench: no tokenizer kernel events (the split tokenizer did not run: %s)' % ks)
  n_gathered = None
  if dist is not None:  # the last step's all-gather saw every rank
    n_gathered = check_gather(gathered[-1], res.bin_count.cpu().numpy(), rank, world)
  if dist is not None:
    t = torch.tensor([el, float(n_tok)], dtype=torch.float64, device=device)
    mx = t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    sm = t.clone()
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    el, tot_tok = float(mx[0]), float(sm[1])
  else:
    tot_tok = float(n_tok)
  if rank != 0:
    dist.destroy_process_group()
    return
  value = tot_tok * args.steps / el
  # roofline of the dominant kernel, the tokenizer's tile scan
  # (lddl::tok5::scan_kernel).  Algorithmic bytes of the
  # scan = the part of the tokenize call's I/O it moves: the corpus read once,
  # 8 B sentence offset read + 4 B token count written per sentence (the 2 B
  # per token id are written by expand_kernel: charged to the whole call in
  # roofline.tokenize_call, never to the scan).  The WordPiece records and
  # entries the scan hands to wp_kernel / expand_kernel are this design's
  # intermediates, not algorithmic (they show in roofline.traffic).  Divided
  # by the scan's HIP-event time inside the call (events on the launch
  # stream; one scan launch per segment of SPLIT_SEG_TILES KiB).
  nl = ks['launches']
  alg_call = sh.nbytes + 12 * sh.n_sent + 2 * n_tok
  alg = (sh.nbytes + 12 * sh.n_sent) / nl
  achieved = alg / (ks['scan_ms'] / nl * 1e-3) / 1e9
  tok_kernels_ms = ks['scan_ms'] + ks['wordpiece_ms'] + ks['expand_ms']
  line = {
      'metric': METRIC, 'value': value, 'unit': 'tokens/s', 'n_gpus': world, 'steps': args.steps,
      'warmup': args.warmup, 'ms_per_step': el * 1e3 / args.steps, 'higher_is_better': True,
      'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u8',
      'data': 'synthetic (%s, %d MB unique tiled x%d per GPU)' % (
          {'code': 'CodeSearchNet-style code', 'wiki': 'Wikipedia-style',
           'wikibooks': 'Wikipedia + Books-style'}[args.corpus], args.unique_mb, reps),
      'config': {'workload': '%s_seq%d_bin%d_%dGB_per_gpu%s' % ({'code': 'codebert', 'wiki': 'bert',
                                                                   'wikibooks': 'bert_wikibooks'}[args.corpus],
                                                                 args.target_seq_length, args.bin_size,
                                                                   round(sh.nbytes / (1 << 30)),
                                                                   '_masking' if args.masking else ''),
                 'target_seq_length': args.target_seq_length, 'bin_size': args.bin_size,
                 'duplicate_factor': args.duplicate_factor, 'vocab': ('codebert_52000/vocab.txt' if code else
                                                                   'bert-base-uncased (lddl/dask/bert/vocab)'),
                 'corpus_bytes_per_gpu': sh.nbytes, 'sentences_per_gpu': sh.n_sent,
                 'partitions_per_gpu': sh.n_part, 'wordpiece_tokens_per_gpu': n_tok,
                 'pairs_per_gpu': res.n_pairs, 'packed_tokens_per_gpu': res.n_tokens,
                 'masked_positions_per_gpu': res.n_masked,
                 'parallelism': 'shard%d' % world, 'gathered_partitions': n_gathered,
                 # the step's row output: spans of the dense ids (what the writer renders from) or materialised rows
                 'rows': 'spans' if res.spans else 'materialize',
                 # steps pipelined pairwise over two streams (pack k beside tokenize k+1)
                 'step_overlap': bool(overlap)},
      'roofline': {'bound': 'hbm', 'kernel': 'lddl::tok5::scan_kernel', 'achieved': achieved, 'peak': HBM_PEAK_GBS,
                   'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS, 'traffic': None,
                   'algorithmic_bytes_per_launch': alg, 'avg_launch_ms': ks['scan_ms'] / nl,
                   'launches_per_step': nl,
                   # the whole tokenize call (scan + WordPiece + expand kernels) against the same bytes
                   'tokenize_call': {'algorithmic_bytes': alg_call, 'kernels_ms': tok_kernels_ms,
                                     'achieved': alg_call / (tok_kernels_ms * 1e-3) / 1e9,
                                     'frac': alg_call / (tok_kernels_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}},
      'tokenize_ms': tk, 'tokenize_kernels_ms': {'scan': ks['scan_ms'], 'wordpiece': ks['wordpiece_ms'],
                                                 'expand': ks['expand_ms']},
      'wordpiece_records_per_gpu': ks['records'], 'tokenizer_fallback_tiles': ks['fallback_tiles'],
      'gen_s': gen_s,
  }
  try:  # device memory left beside the corpus, the tokenizer / packer scratch and the outputs
    free_b, total_b = torch.cuda.mem_get_info(device)
    line['hbm_free_gb'] = round(free_b / 1e9, 1)
    line['hbm_total_gb'] = round(total_b / 1e9, 1)
  except Exception:  # (diagnostic only)
    pass
  # HBM traffic of the tokenize call from the committed PMC passes of this
  # same workload (rocprofv3 cannot run inside the timed process)
  try:
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles', 'traffic.json')) as f:
      tr = json.load(f)
    for e in tr.get('entries', [tr]):
      if (e.get('workload'), e.get('kernel')) == (line['config']['workload'], line['roofline']['kernel']):
        line['roofline']['traffic'] = e['traffic_bytes_per_call']
        line['roofline']['traffic_source'] = e['source']
  except (OSError, ValueError, KeyError):
    pass
  progress(rank, 'timed steps done')
  if args.parquet_parts > 0:
    try:
      line['parquet_writer'] = parquet_sample(args, pk, res, sh, enc)
    except Exception as e:  # (recorded: the headline line still prints)
      line['parquet_writer'] = {'error': '%s: %s' % (type(e).__name__, e)}
  if enc is not None:
    enc.close()
  if fe is not None:
    line['frontend'] = fe
  if fe2 is not None:
    line['frontend_c2'] = fe2
  if not args.no_cpu_baseline and world == 1:  # the host leg (the oracle): rank 0 at N=1 only
    progress(rank, 'cpu baseline')
    try:
      line['cpu_baseline'] = cpu_baseline(args, base, pdo, args.cpu_seconds)
    except Exception as e:  # (recorded: the headline line still prints)
      line['cpu_baseline'] = {'error': '%s: %s' % (type(e).__name__, e)}
    if not args.no_sample_check:  # the oracle as the checker of one full-size partition of the timed run
      try:
        line['cpu_baseline']['sample_check'] = sample_partition_check(args, pk, res, base, pdo, reps, kw['seed'])
      except Exception as e:  # (recorded, never as a pass: identical is absent)
        line['cpu_baseline']['sample_check'] = {'error': '%s: %s' % (type(e).__name__, e)}
  if world == 1 and args.legs and args.legs != 'none':
    # the other BASELINE workloads, after everything above read the headline's
    # results: its packer scratch goes first (a second context beside it would
    # double the tokenizer / packer scratch), its shards stay for the legs on
    # the same corpus
    del res, pk, ntok
    torch.cuda.empty_cache()
    heads = (sh, base, pdo, reps) if args.corpus == 'wiki' else None
    legs = {}
    for name in [x for x in args.legs.split(',') if x]:
      if LEGS[name]['corpus'] != 'wiki' and heads is not None:
        heads = None
        del sh
        torch.cuda.empty_cache()
      try:
        progress(rank, 'leg ' + name)
        legs[name] = run_leg(args, name, local, device, heads if LEGS[name]['corpus'] == 'wiki' else None)
      except Exception as e:  # (recorded: the headline line still prints)
        legs[name] = {'error': '%s: %s' % (type(e).__name__, e)}
      torch.cuda.empty_cache()
    line['legs'] = legs
  print(json.dumps(line), flush=True)
  if dist is not None:
    dist.destroy_process_group()


if __name__ == '__main__':
  main()
