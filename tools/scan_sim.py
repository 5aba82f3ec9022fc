"""CPU model of tok4's WordPiece Bloom scan width (tuning aid, not a test).

For every candidate scan of the WordPiece loop (greedy longest-match-first,
exact vocab, ASCII words <= 24 bytes per piece window), counts the dword
groups evaluated top-down (group k = lengths 4k+1..4k+4) until the match's
group, with and without an "extension" bound: group k+1 is reachable only if
some vocab key longer than 4(k+1) bytes starts with the piece's first
4(k+1) bytes.  The wave runs in lockstep, so the per-iteration cost is the
max over the lanes scanning together (sampled in sets of LANES)."""
import sys, os, random
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def main():
  from lddl_amd import synth
  from lddl_amd.pipeline import VOCAB_BERT
  from oracle.oracle import OracleTokenizer
  vocab = [l.rstrip('\n') for l in open(VOCAB_BERT, encoding='utf-8')]
  keys = set()
  ext = set()
  for w in vocab:
    c = 1 if w.startswith('##') else 0
    b = w[2:].encode() if c else w.encode()
    if not b: continue
    keys.add((c, b))
    for j in range(0, 6):
      if len(b) > 4 * (j + 1): ext.add((c, b[:4 * (j + 1)]))
  maxb = [max(len(b) for (c, b) in keys if c == cc) for cc in (0, 1)]
  c = synth.make_wiki(int(sys.argv[1]) << 20 if len(sys.argv) > 1 else 2 << 20, seed=1)
  ot = OracleTokenizer(VOCAB_BERT)
  base, pruned = [], []
  for si in range(c.n_sent):
    for w in ot.words(c.sentence(si)):
      wb = w.encode()
      if not wb.isascii() or len(wb) > 100: continue
      if len(wb) <= 24 and (0, wb) in keys: continue  # first-probe batch
      s, n, cont = 0, len(wb), 0
      while s < n:
        top = min(n - s, maxb[cont], 24)
        f = 0
        for e in range(min(n, s + maxb[cont]), s, -1):
          if (cont, wb[s:e]) in keys: f = e - s; break
        gt, gf = (top - 1) // 4, ((f - 1) // 4 if f else 0)
        ga = 0
        while ga < 5 and (cont, wb[s:s + 4 * (ga + 1)]) in ext and s + 4 * (ga + 1) < n: ga += 1
        base.append(gt - gf + 1)
        pruned.append(max(min(gt, ga) - gf + 1, 1))
        if not f: break
        s += f; cont = 1
  base, pruned = np.array(base), np.array(pruned)
  lanes = int(os.environ.get('LANES', '32'))
  rng = random.Random(0)
  idx = list(range(len(base)))
  mb, mp = [], []
  for _ in range(2000):
    sel = rng.sample(idx, lanes)
    mb.append(base[sel].max()); mp.append(pruned[sel].max())
  print('scans %d  groups/scan base %.2f pruned %.2f  lockstep max over %d lanes: base %.2f pruned %.2f' % (
      len(base), base.mean(), pruned.mean(), lanes, np.mean(mb), np.mean(mp)))


if __name__ == '__main__':
  main()
