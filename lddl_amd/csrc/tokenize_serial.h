// Serial (one lane per sentence) tokenizer path of tokenize_fallback_kernel
// (the split tokenizer's exact fallback).  Restates oracle/tokenizer_oracle.c (HF tokenizers
// BertNormalizer + BertPreTokenizer + WordPiece, reference call site
// lddl/dask/bert/pretrain.py:79-80).
#pragma once
#include "common.h"
#include "tokenize.h"

namespace lddl {

constexpr int WB_LDS = 64;    // bytes of word buffer per lane held in LDS
constexpr int BLOCK = 256;

// The functions below are host + device: tests/host_serial.cpp builds them
// for the host (g++, AddressSanitizer) over the same tables.
#ifdef __HIP__
// per-lane word buffer: bytes [0, WB_LDS) in LDS, dword-interleaved across
// the block's lanes (byte i of lane t in word [i>>2][t]: conflict-free when
// lanes touch the same i), the rest in a per-lane global overflow slab.
__shared__ uint32_t g_wlds[WB_LDS / 4][BLOCK];

struct LdsWordBuf {
  uint8_t* ovf;  // bytes >= WB_LDS
  __device__ __forceinline__ uint32_t get(int i) const {
    if (i < WB_LDS) return (g_wlds[i >> 2][threadIdx.x] >> ((i & 3) * 8)) & 0xFFu;
    return ovf[i - WB_LDS];
  }
  __device__ __forceinline__ void put(int i, uint32_t v) const {
    if (i < WB_LDS) {  // (a byte-typed LDS store here trips a gfx950 isel bug)
      uint32_t& w = g_wlds[i >> 2][threadIdx.x];
      const int sh = (i & 3) * 8;
      w = (w & ~(0xFFu << sh)) | ((v & 0xFFu) << sh);
    } else {
      ovf[i - WB_LDS] = (uint8_t)v;
    }
  }
};

#endif

// all bytes in one slab (the host build's word buffer)
struct GlobalWordBuf {
  uint8_t* ovf;  // WB_LDS + WB_OVF bytes
  LDDL_HD uint32_t get(int i) const { return ovf[i]; }
  LDDL_HD void put(int i, uint32_t v) const { ovf[i] = (uint8_t)v; }
};

struct SentState {
  int64_t p, e;     // byte cursor / end
  int64_t obase;    // output index of token 0
  int32_t ntok;
};

LDDL_HD void emit(const TokParams& P, SentState& st, uint32_t id) {
  if (st.ntok < P.max_tok) P.out_ids[st.obase + st.ntok] = (uint16_t)id;
  st.ntok++;
}

LDDL_HD int utf8_len(uint32_t b) { return b < 0x80 ? 1 : b >= 0xF0 ? 4 : b >= 0xE0 ? 3 : 2; }
LDDL_HD int utf8_enc_len(uint32_t c) { return c < 0x80 ? 1 : c < 0x800 ? 2 : c < 0x10000 ? 3 : 4; }

template <class WB>
LDDL_HD int put_utf8(const WB& wb, int at, uint32_t c) {
  if (at > WB_LDS + WB_OVF - 4) return 0;  // never reached for words <= 100 chars
  if (c < 0x80) { wb.put(at, c); return 1; }
  if (c < 0x800) { wb.put(at, 0xC0 | (c >> 6)); wb.put(at + 1, 0x80 | (c & 0x3F)); return 2; }
  if (c < 0x10000) {
    wb.put(at, 0xE0 | (c >> 12)); wb.put(at + 1, 0x80 | ((c >> 6) & 0x3F)); wb.put(at + 2, 0x80 | (c & 0x3F));
    return 3;
  }
  wb.put(at, 0xF0 | (c >> 18)); wb.put(at + 1, 0x80 | ((c >> 12) & 0x3F));
  wb.put(at + 2, 0x80 | ((c >> 6) & 0x3F)); wb.put(at + 3, 0x80 | (c & 0x3F));
  return 4;
}

LDDL_HD uint32_t table_entry(const TokParams& P, uint32_t cp) {
  return P.pages[(uint32_t)P.top[cp >> 8] * 256u + (cp & 255u)];
}

// literal [PAD] [UNK] [CLS] [SEP] [MASK] starting at p (byte p is '[')
LDDL_HD int match_special(const uint8_t* s, int64_t p, int64_t e, int* len) {
  if (p + 5 > e) return -1;
  uint32_t c1 = s[p + 1], c2 = s[p + 2], c3 = s[p + 3], c4 = s[p + 4];
  if (c1 == 'P' && c2 == 'A' && c3 == 'D' && c4 == ']') { *len = 5; return 0; }
  if (c1 == 'U' && c2 == 'N' && c3 == 'K' && c4 == ']') { *len = 5; return 1; }
  if (c1 == 'C' && c2 == 'L' && c3 == 'S' && c4 == ']') { *len = 5; return 2; }
  if (c1 == 'S' && c2 == 'E' && c3 == 'P' && c4 == ']') { *len = 5; return 3; }
  if (c1 == 'M' && c2 == 'A' && c3 == 'S' && c4 == 'K' && p + 6 <= e && s[p + 5] == ']') { *len = 6; return 4; }
  return -1;
}

// Exact vocab lookup of (cont, bytes[s, s+len)); h = poly hash of those bytes.
// One 16-byte slot load per probe; keys of <= 8 bytes verify against the
// slot's prefix, longer ones additionally against the 4-aligned pool (all
// dword loads issued together, no per-byte dependent chain).
struct NoFilter {
  LDDL_HD bool operator()(uint64_t) const { return true; }
};

template <class GET, class FILT>
LDDL_HD int probe(const TokParams& P, const GET& get, int s, int len, uint32_t cont, uint64_t h,
                                     const FILT& filt) {
  const uint64_t key = hash_key(h, (uint32_t)len, cont);
  if (!filt(key)) return -1;  // exact negative
  uint32_t idx = (uint32_t)key & P.slot_mask;
  const uint32_t fp = (uint32_t)(key >> 32);
  const uint32_t want = ((uint32_t)len << 16) | (cont << 24) | 0x80000000u;
  uint32_t c0 = 0, c1 = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t b = k < len ? get(s + k) : 0u;
    if (k < 4) c0 |= b << (8 * k); else c1 |= b << (8 * (k - 4));
  }
  for (;;) {
    const uint4 sl = P.slots[idx];
    if (!(sl.y & 0x80000000u)) return -1;
    if (sl.x == fp && (sl.y & 0xFFFF0000u) == want && sl.z == c0 && sl.w == c1) {
      const uint32_t id = sl.y & 0xFFFFu;
      if (len <= 8) return (int)id;
      const uint32_t* v = reinterpret_cast<const uint32_t*>(P.pool + P.voff[id]);
      bool eq = true;
      for (int k = 8; k < len; k += 4) {
        const uint32_t w = v[k >> 2];
        uint32_t cw = 0;
        for (int q = 0; q < 4; ++q) cw |= (k + q < len ? get(s + k + q) : 0u) << (8 * q);
        eq = eq && (w == cw);
      }
      if (eq) return (int)id;
    }
    idx = (idx + 1) & P.slot_mask;
  }
}

// Greedy longest-match-first over bytes [0, nb) of a normalised word.
// EMIT(n, id) is called per piece; returns #pieces, or -1 when some position
// has no match (the caller then emits the single [UNK]).
template <class GET, class EMIT, class FILT = NoFilter>
LDDL_HD int wordpiece_core(const TokParams& P, const GET& get, int nb, const EMIT& emit_fn,
                                              const FILT& filt = FILT()) {
  int s = 0, n = 0;
  uint32_t cont = 0;
  while (s < nb) {
    int e = s + (int)P.maxb[cont];
    if (e > nb) e = nb;
    while (e < nb && e > s && (get(e) & 0xC0u) == 0x80u) --e;
    uint64_t h = 0;
    for (int k = s; k < e; ++k) h = hash_push(h, get(k));
    int id = -1;
    while (e > s) {
      id = probe(P, get, s, e - s, cont, h, filt);
      if (id >= 0) break;
      do { --e; h = hash_pop(h, get(e)); } while (e > s && (get(e) & 0xC0u) == 0x80u);
    }
    if (id < 0) return -1;
    emit_fn(n, (uint32_t)id);
    ++n;
    s = e;
    cont = 1;
  }
  return n;
}

// WordPiece over the buffered normalised word (nb bytes, nch chars).
template <class WB>
__host__ __device__ void wordpiece(const TokParams& P, SentState& st, const WB& wb, int nb, int nch) {
  if (nch > 100) { emit(P, st, P.unk); return; }
  const int32_t mark = st.ntok;
  auto get = [&](int i) { return wb.get(i); };
  auto em = [&](int, uint32_t id) { emit(P, st, id); };
  if (wordpiece_core(P, get, nb, em) < 0) { st.ntok = mark; emit(P, st, P.unk); }
}

// Append one normalised char; keeps each run of ccc>0 chars stably sorted by
// rank (NFD canonical ordering).  Rare path only for chars with rank > 0.
template <class WB>
LDDL_HD void append_char(const TokParams& P, const WB& wb, int& nb, int& nch,
                                            uint32_t c, uint32_t rank, uint32_t& prev_rank, int& run_start) {
  ++nch;
  if (nch > 100) return;  // word becomes [UNK]; stop buffering
  if (rank == 0) { prev_rank = 0; nb += put_utf8(wb, nb, c); return; }
  if (prev_rank == 0) run_start = nb;
  if (prev_rank <= rank) { prev_rank = rank; nb += put_utf8(wb, nb, c); return; }
  // insertion: first char in [run_start, nb) whose rank > rank
  int pos = run_start;
  while (pos < nb) {
    uint32_t b0 = wb.get(pos);
    int l = utf8_len(b0);
    uint32_t cp = b0 < 0x80 ? b0 : (b0 & (0x3Fu >> (l - 1)));
    for (int k = 1; k < l; ++k) cp = (cp << 6) | (wb.get(pos + k) & 0x3Fu);
    if (ent_rank(table_entry(P, cp)) > rank) break;
    pos += l;
  }
  const int l = utf8_enc_len(c);
  for (int k = nb - 1; k >= pos; --k) wb.put(k + l, wb.get(k));
  put_utf8(wb, pos, c);
  nb += l;
}

// One step: the next word (or special token / isolated char) of the sentence.
template <class WB>
__host__ __device__ void step(const TokParams& P, SentState& st, const WB& wb, const uint32_t* ascii_tab) {
  int nb = 0, nch = 0, run_start = 0;
  uint32_t prev_rank = 0;
  const uint8_t* bytes = P.bytes;
  while (st.p < st.e) {
    const uint32_t b = bytes[st.p];
    if (b == '[') {
      int sl;
      const int k = match_special(bytes, st.p, st.e, &sl);
      if (k >= 0) {
        if (nch > 0) break;  // flush the pending word first
        emit(P, st, P.special[k]);
        st.p += sl;
        return;
      }
    }
    uint32_t cp, ent;
    int adv;
    if (b < 0x80) {
      cp = b; adv = 1; ent = ascii_tab[b];
    } else {
      adv = utf8_len(b);
      cp = b & (0x3Fu >> (adv - 1));
      for (int k = 1; k < adv; ++k) cp = (cp << 6) | (bytes[st.p + k] & 0x3Fu);
      if (cp > 0x10FFFF) cp = 0xFFFD;
      ent = table_entry(P, cp);
    }
    const uint32_t kind = ent_kind(ent);
    if (kind == KIND_DROP_T) { st.p += adv; continue; }
    if (kind == KIND_DROP_D) { st.p += adv; prev_rank = 0; continue; }
    if (kind == KIND_MULTI) {
      const uint4 m = P.multi[ent_payload(ent)];
      append_char(P, wb, nb, nch, ent_payload(m.y), ent_rank(m.y), prev_rank, run_start);
      append_char(P, wb, nb, nch, ent_payload(m.z), ent_rank(m.z), prev_rank, run_start);
      if (m.x > 2) append_char(P, wb, nb, nch, ent_payload(m.w), ent_rank(m.w), prev_rank, run_start);
      st.p += adv;
      continue;
    }
    const uint32_t cls = ent_cls(ent);
    if (cls == CLS_SPACE) {
      st.p += adv;
      if (nch > 0) break;
      continue;
    }
    const uint32_t oc = kind == KIND_IDENT ? cp : ent_payload(ent);
    if (cls == CLS_ISOLATE) {
      if (nch > 0) break;  // word ends before the isolated char
      st.p += adv;
      nb = put_utf8(wb, 0, oc);
      nch = 1;
      break;
    }
    append_char(P, wb, nb, nch, oc, ent_rank(ent), prev_rank, run_start);
    st.p += adv;
  }
  if (nch > 0) wordpiece(P, st, wb, nb, nch);
}


}  // namespace lddl
