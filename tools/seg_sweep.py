"""Tokenizer segment-size sweep (GPU box tool): one synthetic corpus, the
split tokenizer at several LDDL_SPLIT_SEG values (tiles of 1 KiB per
segment), min of 3 timed calls each; checks every variant's ids equal the
first one's.
    python tools/seg_sweep.py MB seg1 seg2 ...
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
  mb = int(sys.argv[1])
  segs = [int(x) for x in sys.argv[2:]]
  from lddl_amd import synth
  from lddl_amd.tokenizer import Tokenizer
  corpus = os.environ.get('CORPUS', 'wiki')
  c = synth.make_code(mb << 20, seed=1) if corpus == 'code' else synth.make_wiki(mb << 20, seed=1)
  d = torch.from_numpy(np.concatenate([c.data, np.zeros(16, np.uint8)])).cuda()
  o = torch.from_numpy(c.sent_off).cuda()
  tok = Tokenizer()
  tok.set_timing(True)
  ref = None
  for seg in segs:
    os.environ['LDDL_SPLIT_SEG'] = str(seg)
    ids, ntok, toff = tok.tokenize_device(d, o)
    torch.cuda.synchronize()
    n = int(toff[-1].item())
    h = ids[:n].cpu().numpy()
    same = True
    if ref is None:
      ref = h
    else:
      same = np.array_equal(ref, h)
    times, ks = [], []
    for _ in range(3):
      s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
      s.record()
      tok.tokenize_device(d, o, out_ids=ids, out_ntok=ntok, out_tok_off=toff)
      e.record()
      torch.cuda.synchronize()
      times.append(s.elapsed_time(e))
      ks.append(tok.stats())
    k = ks[int(np.argmin(times))]
    print('seg %8d tiles (%6.0f MB): %.3f ms  %.1f GB/s  scan %.3f wp %.3f finish %.3f (%d launches)  same %s' % (
        seg, seg / 1024, min(times), c.nbytes / min(times) / 1e6, k['scan_ms'], k['wordpiece_ms'], k['expand_ms'],
        k['launches'], same), flush=True)


if __name__ == '__main__':
  main()
