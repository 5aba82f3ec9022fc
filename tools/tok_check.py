"""GPU tokenizer check + timing for the kernel variants (GPU box tool).

    python tools/tok_check.py [MB] [algo ...]   (algo 6: lane tokenizer, 5: split tokenizer, 0: serial path)

Tokenizes a synthetic Wikipedia-style corpus of MB megabytes with each
variant, compares ids / counts with the oracle (first MB only, for speed)
and prints throughput.  LDDL_TOK_DEBUG=1 adds the kernels' phase stamps.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
  mb = int(sys.argv[1]) if len(sys.argv) > 1 else 64
  variants = sys.argv[2:] or ['5']
  from lddl_amd import synth
  from lddl_amd.tokenizer import Tokenizer
  from lddl_amd.pipeline import VOCAB_BERT
  from oracle.oracle import OracleTokenizer, compact
  t0 = time.time()
  c = synth.make_wiki(mb << 20, seed=1)
  if os.environ.get('ASCII') == '1':  # diagnostics: no exception bytes (non-ASCII -> 'x', '[' -> '(')
    c.data[c.data >= 0x80] = ord('x')
    c.data[c.data == ord('[')] = ord('(')
  print('gen %.1fs: %d bytes %d sentences' % (time.time() - t0, c.nbytes, c.n_sent), flush=True)
  d = torch.from_numpy(np.concatenate([c.data, np.zeros(16, np.uint8)])).cuda()
  o = torch.from_numpy(c.sent_off).cuda()
  # NOCHECK=1 (profiling runs): no oracle comparison
  ns_chk = 0 if os.environ.get('NOCHECK') == '1' else int(np.searchsorted(c.sent_off, min(c.nbytes, 4 << 20)))
  oids, ontok = OracleTokenizer(VOCAB_BERT).run(
      c.data, c.sent_off[:ns_chk + 1], 512, nthreads=8)
  for v in variants:
    algo = v
    os.environ['LDDL_TOKENIZE_ALGO'] = algo
    tok = Tokenizer()
    ids, ntok, toff = tok.tokenize_device(d, o)
    torch.cuda.synchronize()
    h_ntok = ntok.cpu().numpy()[:c.n_sent]
    h_toff = toff.cpu().numpy()
    h_ids = ids.cpu().numpy().view(np.uint16)
    bad = np.nonzero(h_ntok[:ns_chk] != ontok)[0]
    nbad_ids = 0
    if len(bad) == 0:
      for i, (a, b) in enumerate(zip([h_ids[h_toff[k]:h_toff[k + 1]] for k in range(ns_chk)],
                                     compact(oids, ontok, c.sent_off[:ns_chk + 1]))):
        if not np.array_equal(a.astype(np.int64), b.astype(np.int64)):
          nbad_ids += 1
          if nbad_ids <= 3:
            print('  ids differ in sentence %d: %r\n   gpu %s\n   ref %s' % (
                i, c.sentence(i)[:200], a[:40].tolist(), b[:40].tolist()))
    else:
      for i in bad[:3]:
        print('  ntok differs in sentence %d (%d vs %d): %r' % (i, h_ntok[i], ontok[i], c.sentence(i)[:200]))
    ok = len(bad) == 0 and nbad_ids == 0
    ntoks = int(h_ntok.sum())
    times, ks = [], []
    if algo in ('5', '6'):
      tok.set_timing(True)
    for _ in range(3):
      s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
      s.record()
      tok.tokenize_device(d, o, out_ids=ids, out_ntok=ntok, out_tok_off=toff)
      e.record()
      torch.cuda.synchronize()
      times.append(s.elapsed_time(e))
      if algo in ('5', '6'):
        ks.append(tok.stats())
    ms = min(times)
    if ks:
      print('  per kernel (min of 3): scan %.3f  wordpiece %.3f  finish %.3f ms; %d records, %d fallback tiles' % (
          min(k['scan_ms'] for k in ks), min(k['wordpiece_ms'] for k in ks), min(k['expand_ms'] for k in ks),
          ks[0]['records'], ks[0]['fallback_tiles']))
    print('variant %s: parity(%d sents) %s (ntok bad %d, ids bad %d)  %.3f ms  %.1f GB/s  %.2f Gtok/s' % (
        v, ns_chk, 'OK' if ok else 'FAIL', len(bad), nbad_ids, ms, c.nbytes / ms / 1e6, ntoks / ms / 1e6),
          flush=True)
    tok.close()


if __name__ == '__main__':
  main()
