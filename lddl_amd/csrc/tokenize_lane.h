// Lane tokenizer (tok6): one lane per tile of sentences, one byte of its
// stream per iteration, greedy longest-match WordPiece as a walk of a
// double-array trie (tok_tables.h build_trie).  The per-lane logic lives here
// as host + device functions: tokenize_lane.hip runs it as a wave of 64 lanes
// on the GPU, tests/host_lane.cpp emulates such a wave on the host (g++,
// AddressSanitizer) over the same tables.
//
// Contract: lddl_tokenize (include/lddl_amd.h) -- the ids HF tokenizers'
// BertNormalizer / BertPreTokenizer / WordPiece give behind
// tokenizer.tokenize(s, max_length=512, truncation=True) at
// lddl/dask/bert/pretrain.py:79-80 (restated in oracle/tokenizer_oracle.c).
//
// Why: the tile tokenizer (tok5) deals a tile's units to lanes, which
// costs ~350 instructions of bookkeeping per unit step plus a WordPiece
// record per missed word (~2000 instructions per record in its Bloom-scan
// WordPiece kernel).  Here a lane walks its own bytes: per byte a class
// lookup, one trie load and a few selects; a word's pieces come out of the
// same walk (the trie answers "longest vocab key from here"), so whole-word
// hits and WordPiece are one code path and no record or entry is written.
//
// Per lane and iteration (modes M_*):
//   SCAN  at a unit boundary: spaces / dropped controls skipped, a literal
//         [PAD] [UNK] [CLS] [SEP] [MASK] emitted, an ASCII word char or
//         isolate starts a WORD walk in the same iteration; a non-ASCII byte
//         asks for the slow path (SLOW).
//   WORD  feeds the byte at p to the trie (its class table gives the
//         normalised byte: A-Z -> a-z) and looks at byte p+1: the word ends at
//         a space / isolate / '[' / the sentence end (its last piece is
//         emitted and a following space consumed), a non-ASCII or dropped
//         byte restarts the word on the slow path.  When the walk cannot
//         extend, the last accepting prefix is a piece: it is emitted and the
//         walk restarts from the "##" root at its end (back-tracking p);
//         without one the word is [UNK] (its pieces rolled back) and SKIP
//         runs to its end.
//   BUF   the same walk over a normalised word the slow path left in the
//         lane's ring (up to RING_BYTES bytes).
//   SLOW  waiting for the wave's batched slow pass (lane_slow): the exact
//         serial normaliser of tokenize_serial.h over the raw bytes (code
//         point tables, multi-char expansions, canonical reordering), which
//         leaves a word in the buffer (BUF), emits a special or [UNK], or
//         hands the position back to SCAN.
// Sentence ids are staged at the sentence's byte offset in the segment
// (no code point normalises to more chars than its UTF-8 bytes, so a
// sentence never has more tokens than bytes; UniTables::lane_ok);
// tokenize_lane.hip compacts them into the dense CSR output.
#pragma once
#include "common.h"
#include "tokenize.h"
#include "tokenize_serial.h"

namespace lddl {
namespace tok6 {

constexpr int RING_SLOTS = 4;                 // 16-B chunks of a lane's byte ring (LDS)
constexpr int RING_BYTES = 16 * RING_SLOTS;   // also the slow path's word buffer
constexpr int LANE_BATCH = 64;                // tiles handed to a wave per counter round trip
constexpr int REFILL_EVERY = 16;              // iterations between ring refills (a lane eats <= 1 B / iteration)
constexpr int SLOW_BATCH = 8;                 // waiting lanes that trigger the wave's slow pass
constexpr int SLOW_AGE = 24;                  // ... or iterations the oldest has waited
constexpr int WALK_STEPS = 4;                 // trie steps a lane may take per iteration

enum : uint32_t { M_IDLE = 0, M_NEED, M_TILE, M_TILE2, M_SCAN, M_WORD, M_BUF, M_SKIP, M_SLOW };
enum : uint32_t { SL_UNIT = 1, SL_WORD = 2, SL_SKIPCH = 3 };

struct LaneState {
  uint32_t mode, slow;
  uint32_t iso, spec;     // the word is one isolated char; the sentence emitted [CLS] / [SEP]
  int64_t t;              // tile
  int64_t s, sb;          // sentence, one past the tile's last
  int64_t tb16;           // 16-aligned base of the tile's bytes: positions below are relative to it
  int64_t obase;          // staging index of the sentence's token 0 (M_TILE: the tile's first byte)
  int64_t sa1, sa2;       // sent_off[s + 1], sent_off[s + 2] as of the previous iteration: every
                          // iteration loads them for the next, so a sentence start never waits
                          // on a load it issued (and no branch merge copies a pending load)
  int32_t p, se;          // byte cursor, sentence end
  int32_t w0, ps, la;     // word start, piece start, end of the longest accepted piece (< 0: none);
                          // BUF: buffer indices
  int32_t nt, wt;         // tokens of the sentence, tokens before the word
  uint32_t node, nbase, laid;  // trie node, its children's base, the accepted piece's id
  int32_t bi, bn;         // BUF: cursor, word bytes
  int32_t rlo, rhi;       // ring: chunks [rhi - RING_SLOTS, rhi) of (p >> 4) granularity are loaded
};


template <class E>
LDDL_HD void emit_tok(LaneState& L, const E& en, uint32_t id) {
  if (L.nt < en.P.max_tok) en.put_tok(L.obase + L.nt, id);
  ++L.nt;
}

// the buffer view append_char / put_utf8 (tokenize_serial.h) write through
template <class E>
struct LaneWB {
  const E* en;
  LDDL_HD uint32_t get(int i) const { return i < RING_BYTES ? en->bget(i) : 0u; }
  LDDL_HD void put(int i, uint32_t v) const {
    if (i < RING_BYTES) en->bput(i, v);
  }
};

// The wave's slow pass for one waiting lane.
template <class E>
LDDL_HD void lane_slow(LaneState& L, const E& en) {
  const TokParams& P = en.P;
  const int64_t base = L.tb16;
  auto entry = [&](uint32_t b, int64_t a, int* adv) -> uint32_t {
    if (b < 0x80) { *adv = 1; return en.asc(b); }
    const int n = utf8_len(b);
    uint32_t cp = b & (0x3Fu >> (n - 1));
    for (int k = 1; k < n; ++k) cp = (cp << 6) | (en.raw(a + k) & 0x3Fu);
    if (cp > 0x10FFFF) cp = 0xFFFD;
    *adv = n;
    return cp < 0x10000u ? P.bmp[cp] : table_entry(P, cp);
  };
  if (L.slow == SL_SKIPCH) {  // SKIP at a non-ASCII char: does it end the [UNK] word?
    int adv = 1;
    const uint32_t e = entry(en.raw(base + L.p), base + L.p, &adv);
    const uint32_t kind = ent_kind(e), cls = ent_cls(e);
    const bool brk = kind != KIND_DROP_T && kind != KIND_DROP_D && kind != KIND_MULTI &&
                     (cls == CLS_SPACE || cls == CLS_ISOLATE);
    if (brk) {
      L.mode = M_SCAN;
    } else {
      L.p += adv;
      L.mode = M_SKIP;
    }
    return;
  }
  const LaneWB<E> wb{&en};
  const int32_t q0 = L.slow == SL_WORD ? L.w0 : L.p;
  int32_t q = q0;
  int nb = 0, nch = 0, run_start = 0;
  uint32_t prev_rank = 0;
  while (q < L.se) {
    const uint32_t b = en.raw(base + q);
    if (nch == 0 && q > q0 && b < 0x80) break;  // only skipped chars so far: back to the fast path
    if (b == '[') {
      int sl = 0;
      const int k = match_special(P.bytes, base + q, base + L.se, &sl);
      if (k >= 0) {
        if (nch > 0) break;
        emit_tok(L, en, P.special[k]);
        if ((k == 2 || k == 3) && L.nt <= P.max_tok) L.spec = 1;
        q += sl;
        L.p = q;
        L.mode = M_SCAN;
        return;
      }
    }
    int adv = 1;
    const uint32_t ent = entry(b, base + q, &adv);
    const uint32_t kind = ent_kind(ent);
    if (kind == KIND_DROP_T) { q += adv; continue; }
    if (kind == KIND_DROP_D) { q += adv; prev_rank = 0; continue; }
    if (kind == KIND_MULTI) {
      const uint4 m = P.multi[ent_payload(ent)];
      append_char(P, wb, nb, nch, ent_payload(m.y), ent_rank(m.y), prev_rank, run_start);
      append_char(P, wb, nb, nch, ent_payload(m.z), ent_rank(m.z), prev_rank, run_start);
      if (m.x > 2) append_char(P, wb, nb, nch, ent_payload(m.w), ent_rank(m.w), prev_rank, run_start);
      q += adv;
      continue;
    }
    const uint32_t cls = ent_cls(ent);
    if (cls == CLS_SPACE) {
      q += adv;
      if (nch > 0) break;
      continue;
    }
    uint32_t cp;
    if (b < 0x80) {
      cp = b;
    } else {
      const int n = adv;
      cp = b & (0x3Fu >> (n - 1));
      for (int k = 1; k < n; ++k) cp = (cp << 6) | (en.raw(base + q + k) & 0x3Fu);
      if (cp > 0x10FFFF) cp = 0xFFFD;
    }
    const uint32_t oc = kind == KIND_IDENT ? cp : ent_payload(ent);
    if (cls == CLS_ISOLATE) {
      if (nch > 0) break;
      q += adv;
      nb = put_utf8(wb, 0, oc);
      nch = 1;
      break;
    }
    append_char(P, wb, nb, nch, oc, ent_rank(ent), prev_rank, run_start);
    q += adv;
  }
  L.p = q;
  if (nch == 0) {  // reached the sentence end, or back to the fast path
    L.mode = M_SCAN;
    return;
  }
  if (L.slow == SL_UNIT) L.wt = L.nt;
  if (nch > 100) {  // max_input_chars_per_word
    emit_tok(L, en, P.unk);
    L.mode = M_SCAN;
    L.rlo = L.rhi = L.p >> 4;  // (the word's bytes went through the ring's storage)
    return;
  }
  if (nb > RING_BYTES) {  // does not fit the buffer: the exact serial kernel re-runs the tile
    en.abort_tile(L);
    L.mode = M_NEED;
    return;
  }
  L.bi = 0;
  L.bn = nb;
  L.ps = 0;
  L.la = -1;
  L.node = 0;
  L.nbase = en.Q.rbase[0];
  L.mode = M_BUF;
}

template <class E>
LDDL_HD void sentence_end(LaneState& L, const E& en) {
  const TokParams& P = en.P;
  en.put_ntok(L.s, L.nt < P.max_tok ? L.nt : P.max_tok, L.spec);
  ++L.s;
  if (L.s >= L.sb) {
    L.mode = M_NEED;
    return;
  }
  L.p = L.se;  // (a sentence cut at max_tok ends early)
  const int32_t ss = L.se;
  L.se = (int32_t)(L.sa2 - L.tb16);  // (sent_off[s + 1] of the new s)
  L.nt = 0;
  L.spec = 0;
  L.obase = L.tb16 - en.Q.segb + ss;
}

// the tile's first sentence in two iterations: M_TILE has s, sb and the
// tile's first byte offset (obase) from the wave's hand-out; M_TILE2 finds
// sent_off[s + 1] in sa1 (loaded at the end of M_TILE's iteration)
template <class E>
LDDL_HD void tile_start(LaneState& L, const E& en) {
  if (L.mode == M_TILE) {
    if (L.s >= L.sb) {
      L.mode = M_NEED;
      return;
    }
    const int64_t a = L.obase;
    L.tb16 = a & ~(int64_t)15;
    L.p = (int32_t)(a - L.tb16);
    L.rlo = L.rhi = L.p >> 4;
    L.mode = M_TILE2;
    return;
  }
  L.se = (int32_t)(L.sa1 - L.tb16);
  L.nt = 0;
  L.spec = 0;
  L.obase = L.tb16 - en.Q.segb + L.p;
  L.mode = M_SCAN;
}

// literal special token at ring position p (byte p is '[') within [p, se)
template <class E>
LDDL_HD int special_at(const E& en, int32_t p, int32_t se, int32_t* len) {
  if (p + 5 > se) return -1;
  const uint32_t c1 = en.rbyte(p + 1), c2 = en.rbyte(p + 2), c3 = en.rbyte(p + 3), c4 = en.rbyte(p + 4);
  const uint32_t w = c1 | c2 << 8 | c3 << 16 | c4 << 24;
  *len = 5;
  if (w == 0x5D444150u) return 0;  // PAD]
  if (w == 0x5D4B4E55u) return 1;  // UNK]
  if (w == 0x5D534C43u) return 2;  // CLS]
  if (w == 0x5D504553u) return 3;  // SEP]
  if (w == 0x4B53414Du && p + 6 <= se && en.rbyte(p + 5) == ']') {  // MASK]
    *len = 6;
    return 4;
  }
  return -1;
}

template <class E>
LDDL_HD void lane_step(LaneState& L, const E& en) {
  const TokParams& P = en.P;
  const uint32_t mode = L.mode;
  const bool buf = mode == M_BUF;
  // every lane reads its ring at the cursor and one byte past it and issues
  // one trie load, whatever its mode (lanes with nothing to feed load entry
  // 0): branch-free up to the trie entry, which is then used whole
  int32_t q = buf ? L.bi : L.p;
  const uint32_t b = en.rbyte(q), c = en.ctab(b), cls = c >> 8;
  const uint32_t c2 = en.ctab(en.rbyte(q + 1)) >> 8;
  const int32_t need_scan = L.p + 6 < L.se ? L.p + 6 : L.se - 1;  // (a special's bytes)
  const int32_t need_word = q + 1 < L.se ? q + 1 : q;
  const bool av = ((mode == M_SCAN ? need_scan : need_word) >> 4) < L.rhi;
  const bool scan = mode == M_SCAN && L.p < L.se && L.nt < P.max_tok && av;
  bool startw = scan && (cls == LANE_CW || cls == LANE_CI || cls == LANE_CLB);
  int32_t splen = 0;
  int spk = -1;
  if (startw && cls == LANE_CLB) {  // '[': a literal special, else an isolate
    spk = special_at(en, L.p, L.se, &splen);
    if (spk >= 0) startw = false;
  }
  const bool walk = buf || (mode == M_WORD && av) || startw;
  const uint32_t nbase = startw ? en.Q.rbase[0] : L.nbase;
  const uint32_t lb = buf ? b : (c & 0xFFu);
  const uint32_t idx = walk ? nbase + lb : 0u;
  const uint2 t = en.trie(idx);
  if (mode == M_TILE || mode == M_TILE2) {
    tile_start(L, en);
  } else if (mode == M_SKIP) {
    if (L.p >= L.se) {
      L.mode = M_SCAN;
    } else if ((L.p >> 4) < L.rhi) {
      if (cls == LANE_CW || cls == LANE_CDR) {
        ++L.p;
      } else if (cls == LANE_CNA) {
        L.slow = SL_SKIPCH;
        L.mode = M_SLOW;
      } else {
        L.mode = M_SCAN;
      }
    }
  } else if (mode == M_SCAN) {
    if (L.p >= L.se || L.nt >= P.max_tok) {
      sentence_end(L, en);
    } else if (!av) {
      // (ring not loaded yet)
    } else if (cls == LANE_CSP || cls == LANE_CDR) {
      ++L.p;
    } else if (cls == LANE_CNA) {
      L.slow = SL_UNIT;
      L.mode = M_SLOW;
    } else if (spk >= 0) {
      emit_tok(L, en, P.special[spk]);
      if ((spk == 2 || spk == 3) && L.nt <= P.max_tok) L.spec = 1;
      L.p += splen;
    } else {  // a word (or an isolated char) starts at p; its first byte is fed below
      L.w0 = L.ps = L.p;
      L.wt = L.nt;
      L.node = 0;
      L.nbase = nbase;
      L.la = -1;
      L.iso = cls != LANE_CW ? 1u : 0u;
      L.mode = M_WORD;
    }
  } else if (mode == M_WORD && !av) {
    const int32_t keep = L.la >= 0 ? L.la : q;
    if (L.rhi - (keep >> 4) >= RING_SLOTS) {  // the piece outgrew the ring: the slow path
      L.nt = L.wt;
      L.slow = SL_WORD;
      L.mode = M_SLOW;
    }
  }
  if (walk) {
    // up to WALK_STEPS trie steps while the word goes on (one dependent trie
    // load each); the iteration's one emit, if any, comes after the steps (a
    // store in between would make the next step's wait include it: vmcnt
    // counts in order)
    uint2 te = t;
    uint32_t ti = idx, c2n = c2;
    bool ok, more, slowish, space;
    for (int j = 1;; ++j) {
      more = slowish = space = false;
      if (buf) {
        more = q + 1 < L.bn;
      } else if (q + 1 < L.se) {
        space = c2n == LANE_CSP;  // (consumed with the word's end)
        if (!L.iso) {
          more = c2n == LANE_CW;
          slowish = c2n == LANE_CNA || c2n == LANE_CDR;
        }
      }
      ok = trie_check(te) == L.node;
      if (!ok) break;
      L.node = ti;
      L.nbase = trie_base(te);
      ++q;
      if (trie_accept(te)) {
        L.la = q;
        L.laid = trie_id(te);
      }
      if (slowish || !more || j == WALK_STEPS) break;
      if (!buf && ((q + 1 < L.se ? q + 1 : q) >> 4) >= L.rhi) break;  // (ring: the next iteration)
      const uint32_t bq = en.rbyte(q);
      c2n = en.ctab(en.rbyte(q + 1)) >> 8;
      ti = L.nbase + (buf ? bq : (en.ctab(bq) & 0xFFu));
      te = en.trie(ti);
    }
    if (ok && slowish) {  // the word goes on with a char the fast path does not model
      L.nt = L.wt;
      L.slow = SL_WORD;
      L.mode = M_SLOW;
    } else if (ok && more) {  // (steps used up, or the ring's next chunk not loaded yet)
      if (buf) L.bi = q;
      else L.p = q;
    } else {
      // the walk stopped at q: the word ends there (ok) or no key extends [ps, q] (!ok)
      bool done = false;
      uint32_t eid = P.unk;
      if (ok && !buf && q - L.w0 > 100) {  // max_input_chars_per_word (an ASCII word: chars = bytes)
        L.nt = L.wt;
        done = true;
      } else if (ok && L.la == q) {
        eid = L.laid;
        done = true;
      } else if (L.la >= 0) {  // the longest piece from ps, then "##" pieces from its end
        eid = L.laid;
        q = L.ps = L.la;
        L.la = -1;
        L.node = 1;
        L.nbase = en.Q.rbase[1];
        if (buf) L.bi = q;
        else L.p = q;
      } else {  // no piece: the word is [UNK]
        L.nt = L.wt;
        if (ok || buf || L.iso) {
          done = true;
          if (!ok && L.iso) q = L.w0 + 1;
        } else {
          L.p = q;
          L.mode = M_SKIP;
        }
      }
      emit_tok(L, en, eid);
      if (done) {
        L.mode = M_SCAN;
        if (buf) L.rlo = L.rhi = L.p >> 4;  // (the buffer held the ring's bytes)
        else L.p = q + ((ok && space) ? 1 : 0);
      }
    }
  }
  const int64_t n = P.n_sent;
  L.sa1 = en.soff(L.s + 1 <= n ? L.s + 1 : n);
  L.sa2 = en.soff(L.s + 2 <= n ? L.s + 2 : n);
}

}  // namespace tok6
}  // namespace lddl
