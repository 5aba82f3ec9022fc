"""lddl_bin on the GPU: time and effective HBM rate of the standalone length
binning (binning.py:63-93) at bench scale, and its result against a stable
sort of the reference's bin ids.  Algorithmic bytes per row: the int64
length read by both passes (16 B) + the int64 row index written (8 B).
  python tools/bin_check.py [ROWS_M] [BIN_SIZE] [NBINS]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
  rows = int(float(sys.argv[1]) * 1e6) if len(sys.argv) > 1 else 100_000_000
  bin_size = int(sys.argv[2]) if len(sys.argv) > 2 else 64
  nbins = int(sys.argv[3]) if len(sys.argv) > 3 else 8
  from lddl_amd.pipeline import Packer, VOCAB_BERT, bin_rows
  pk = Packer(VOCAB_BERT, 0)
  g = torch.Generator(device='cuda').manual_seed(1)
  nt = torch.randint(1, bin_size * nbins + 1, (rows,), generator=g, device='cuda', dtype=torch.int64)
  perm, cnt = bin_rows(pk.tok, nt, bin_size, nbins)  # warm
  torch.cuda.synchronize()
  ts = []
  for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    perm, cnt = bin_rows(pk.tok, nt, bin_size, nbins)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
  ms = min(ts)
  b = torch.clamp(torch.div(nt - 1, bin_size, rounding_mode='floor'), max=nbins - 1)
  ok = bool(torch.equal(perm, torch.sort(b, stable=True).indices)) and bool(
      torch.equal(cnt, torch.bincount(b, minlength=nbins)))
  alg = 24 * rows
  print(json.dumps({'rows': rows, 'bin_size': bin_size, 'nbins': nbins, 'ms': ms, 'ms_all': ts,
                    'algorithmic_bytes': alg, 'GB_per_s': alg / (ms * 1e-3) / 1e9, 'identical': ok}))


if __name__ == '__main__':
  main()
