"""Probe: how much of the packer + materialise can hide behind the tokenizer
when the two run on separate streams (two contexts, so no shared scratch).
Times tokenize alone, pack+materialise alone and both issued together from two
host threads, on the bench corpus (default 10 GB per GPU to leave room for the
second context).  Diagnostic only; not part of the product path.
  python tools/overlap_probe.py [--corpus-gb 10]
"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
  if '--corpus-gb' not in sys.argv:
    sys.argv += ['--corpus-gb', '10']
  args = bench.parse()
  device = torch.device('cuda', 0)
  torch.cuda.set_device(device)
  from lddl_amd.pipeline import Packer, VOCAB_BERT
  sh, base, pdo, reps, _ = bench.build_shards(args, 0, device)
  pk1 = Packer(VOCAB_BERT, device=0)
  pk2 = Packer(VOCAB_BERT, device=0)
  kw = dict(target_seq_length=args.target_seq_length, short_seq_prob=0.1, duplicate_factor=args.duplicate_factor,
            seed=args.seed, bin_size=args.bin_size)
  s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
  ids2, ntok2, toff2 = pk2.tokenize(sh, stream=s2)
  pk2.pack(sh, ids2, ntok2, toff2, stream=s2, **kw)
  pk1.tokenize(sh, stream=s1)
  torch.cuda.synchronize()

  def tok():
    pk1.tokenize(sh, stream=s1)
    s1.synchronize()

  def pack():
    pk2.pack(sh, ids2, ntok2, toff2, stream=s2, **kw)
    s2.synchronize()

  def timed(fns, reps=3):
    out = []
    for _ in range(reps):
      torch.cuda.synchronize()
      t0 = time.perf_counter()
      th = [threading.Thread(target=f) for f in fns]
      for t in th:
        t.start()
      for t in th:
        t.join()
      torch.cuda.synchronize()
      out.append((time.perf_counter() - t0) * 1e3)
    return min(out), out

  a = timed([tok])
  b = timed([pack])
  c = timed([tok, pack])
  print('tokenize alone  %.1f ms %s' % (a[0], [round(x, 1) for x in a[1]]), flush=True)
  print('pack+mat alone  %.1f ms %s' % (b[0], [round(x, 1) for x in b[1]]), flush=True)
  print('both, 2 streams %.1f ms %s (sum %.1f)' % (c[0], [round(x, 1) for x in c[1]], a[0] + b[0]), flush=True)


if __name__ == '__main__':
  main()
