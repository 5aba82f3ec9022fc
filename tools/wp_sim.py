"""CPU model of tok4's WordPiece probe chains (tuning aid, not a test).

Builds the v4 vocab table + Bloom filter exactly as capi.hip does (common.h
vhash), then replays greedy longest-match-first on the words of a synthetic
corpus and reports, per word, the number of bucket probes on its critical path
(one per Bloom-positive candidate, +1 per extra bucket when a key is
displaced), and per 1 KiB tile the max over its words."""
import sys, os, collections
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
M = 0xFFFFFFFF
def vmix(h, d):
  h ^= d; return (((h << 5) | (h >> 27)) & M) * 0x85EBCA77 & M
def vfinal(h, ln, cont):
  h ^= (ln * 0x9E3779B9 & M) ^ (0x7F4A7C15 if cont else 0)
  h ^= h >> 15; h = h * 0x2C1B3C6D & M; h ^= h >> 12; h = h * 0x297A2D39 & M; h ^= h >> 15
  return h
def vhash(b, cont):
  l = min(len(b), 24); q, r = l >> 2, l & 3
  d = b[:24] + b'\0' * 28
  h = 0x1B873593
  for k in range(q): h = vmix(h, int.from_bytes(d[4*k:4*k+4], 'little'))
  if r: h = vmix(h, int.from_bytes(d[4*q:4*q+4], 'little') & ((1 << (8*r)) - 1))
  return vfinal(h, len(b), cont)

def main():
  from lddl_amd import synth
  from lddl_amd.pipeline import VOCAB_BERT
  from oracle.oracle import OracleTokenizer
  vocab = [l.rstrip('\n') for l in open(VOCAB_BERT, encoding='utf-8')]
  V = len(vocab)
  keys = {}
  for i, w in enumerate(vocab):
    c = 1 if w.startswith('##') else 0
    b = w[2:].encode() if c else w.encode()
    if b: keys[(c, b)] = i
  nbk = 1
  while nbk < V * int(os.environ.get("BKX", "1")): nbk <<= 1
  table = [[] for _ in range(nbk)]
  home = {}
  bloom = [0] * 8192
  for (c, b), i in keys.items():  # insertion in vocab order (dict keeps it)
    h = vhash(b, c)
    bloom[h >> 19] |= (1 << (h & 31)) | (1 << ((h >> 5) & 31))
    k = h & (nbk - 1); d = 0
    while len(table[k]) >= 2: k = (k + 1) & (nbk - 1); d += 1
    table[k].append((c, b)); home[(c, b)] = d
  maxb = [max(len(b) for (c, b) in keys if c == cc) for cc in (0, 1)]
  def bloom_ok(h):
    bb = (1 << (h & 31)) | (1 << ((h >> 5) & 31)); return bloom[h >> 19] & bb == bb
  K = int(os.environ.get('K', '1'))
  def chain(word):  # probes on the critical path of one word (ASCII, normalised)
    s, n, probes, pieces = 0, len(word), 0, 0
    cont = 0
    first = True
    while s < n:
      e = min(n, s + maxb[cont])
      pos = []  # Bloom-positive candidate ends, longest first
      while e > s:
        if bloom_ok(vhash(word[s:e], cont)): pos.append(e)
        e -= 1
      hit = None
      for j, e in enumerate(pos):
        if (cont, word[s:e]) in keys: hit = (j, e); break
      if first and pos and pos[0] == n and hit and hit[0] == 0 and n <= 24 and home[(0, word)] == 0:
        pass  # batched first probe (prep), off the queue
      else:
        if hit is None: return probes + (len(pos) + K - 1) // K, -1
        probes += hit[0] // K + 1 + (0 if os.environ.get("NOHOME") else home[(cont, word[s:hit[1]])])
      first = False
      pieces += 1; s = hit[1]; cont = 1
    return probes, pieces
  c = synth.make_wiki(int(sys.argv[1]) << 20 if len(sys.argv) > 1 else 2 << 20, seed=1)
  ot = OracleTokenizer(VOCAB_BERT)
  tile_max = collections.defaultdict(int); tile_sum = collections.defaultdict(int)
  hist = collections.Counter()
  for si in range(c.n_sent):
    t = (c.sent_off[si] - c.sent_off[0]) >> 10
    for w in ot.words(c.sentence(si)):
      wb = w.encode()
      if not wb.isascii() or len(w) > 100: continue
      p, _ = chain(wb)
      hist[p] += 1
      tile_max[t] = max(tile_max[t], p); tile_sum[t] += p
  tot = sum(hist.values())
  print('words', tot, 'probes/word %.3f' % (sum(k * v for k, v in hist.items()) / tot))
  print('chain histogram', sorted(hist.items())[:20])
  mx = np.array(list(tile_max.values())); sm = np.array(list(tile_sum.values()))
  print('per tile: max chain mean %.2f p50 %d p90 %d max %d; queue probes/64 lanes mean %.2f' % (
      mx.mean(), np.percentile(mx, 50), np.percentile(mx, 90), mx.max(), (sm / 64).mean()))

if __name__ == '__main__':
  main()
