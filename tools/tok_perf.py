"""Quick tokenize throughput probe on the GPU box (not the bench)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from lddl_amd import synth
from lddl_amd.tokenizer import Tokenizer
mb = int(sys.argv[1]) if len(sys.argv) > 1 else 128
t0 = time.time(); c = synth.make_wiki(mb << 20, seed=1); print('gen %.1fs' % (time.time() - t0), flush=True)
tok = Tokenizer()
d = torch.from_numpy(np.concatenate([c.data, np.zeros(16, np.uint8)])).cuda()
o = torch.from_numpy(c.sent_off).cuda()
ids, ntok = tok.tokenize_device(d, o)
torch.cuda.synchronize()
ntoks = int(ntok.sum())
print('n_sent', c.n_sent, 'max sent bytes', int(np.diff(c.sent_off).max()))
for max_tok in [512, 512, 1, 4]:
  s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  s.record(); tok.tokenize_device(d, o, max_tok=max_tok, out_ids=ids, out_ntok=ntok); e.record(); torch.cuda.synchronize()
  ms = s.elapsed_time(e)
  print('max_tok %d: bytes %d tokens %d  %.3f ms  %.2f GB/s  %.3f Gtok/s  B/tok %.2f' % (max_tok, c.nbytes, ntoks, ms, c.nbytes / ms / 1e6, ntoks / ms / 1e6, c.nbytes / ntoks), flush=True)
