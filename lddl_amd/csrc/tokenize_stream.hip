// Tokenizer v4 (default): one WAVE per sentence-aligned tile, every wave
// independent (no workgroup barrier after the prologue), persistent grid.
//
// Same contract and results as tokenize_tile.hip / tokenize.hip (reference:
// HF tokenizers' BertNormalizer / BertPreTokenizer / WordPiece behind
// tokenizer.tokenize(s, max_length=512, truncation=True),
// lddl/dask/bert/pretrain.py:79-80; restated in oracle/tokenizer_oracle.c).
//
// Tile t = the sentences whose first byte lies in [t*1KiB, (t+1)*1KiB)
// (tile_bounds_kernel).  A wave owns a tile; its window is the 16-byte
// aligned span of those sentences, <= 2 KiB, 32 bytes per lane.
//
//  1 bytes    two 16-B loads per lane, raw copy in LDS.  A 256-entry class
//             table gives per-lane bit masks (word char, isolate, space, char
//             start, dirty, exception) and the normalised bytes IN PLACE
//             (ASCII lower-cased, dropped chars -> 0xFF filler).  Exceptions
//             (non-ASCII lead bytes, '[') run a short loop: literal specials on
//             the raw text, the per-code-point table for non-ASCII chars; an
//             output longer than its input leaves an expansion marker
//             (0xFD, index) resolved in step 3.
//  2 units    unit starts = isolate chars, specials, and word chars not
//             preceded by a word char (fillers count as word chars, so dropped
//             chars are transparent, and every sentence start breaks); one wave
//             scan -> unit list (position, sentence).
//  3 prep     span of each unit (next break bit); dirty spans compacted /
//             expanded into a side buffer; specials and >100-char words done.
//  4 WordPiece greedy longest-match-first on a per-wave work queue, every
//             lane one vocab probe per step: candidate = its first 24 bytes as
//             6 dwords from LDS, hash, LDS Bloom filter (exact negatives cost no
//             memory access), one 64-B bucket load for the rest; pieces stored
//             at the unit's raw position (#pieces <= #raw bytes of the unit).
//  5 output   segmented wave scan of piece counts by sentence, ids written to
//             their final slots, per-sentence counts.
// Tiles it does not model (window > 2 KiB, > 64 sentences, > 256 units, side
// buffer or marker overflow, ccc>0 survivors needing canonical reordering)
// are listed and re-run by tokenize_fallback_kernel (exact serial path).
#include "common.h"
#include "tokenize.h"
#include "wave.h"
#include "tokenize_serial.h"

namespace lddl {
namespace tok4 {

// Geometry of one wave's tile: H = 1 (1 KiB of sentence starts, 2 KiB
// window, 32 B per lane) or H = 2 (two 1 KiB tiles as one: 4 KiB window as two
// 2 KiB halves, twice the units per WordPiece pass -- the pass's serial
// chain is the longest word's, so its lanes fill up; half the waves per CU)
template <int H>
struct Geo {
  static constexpr int CAP = 2048 * H;              // window bytes (32 per lane per half)
  static constexpr int DCAP = 256 * H;              // side buffer for dirty words
  static constexpr int NBUF = CAP + DCAP + 64;      // + over-read pad of the candidate loads
  static constexpr int UCAP = 256 * H;              // units per round
  static constexpr int NSCAP = 64 * H;              // sentences per tile
  static constexpr int XCAP = 32 * H;               // expansion markers per tile
  static constexpr int MPCAP = CAP / 2 - UCAP * 2;  // multi-piece buffer entries (u16) per round
  // work entry: unit | window position << UB | byte length << LSH
  static constexpr int UB = 7 + H, SB = 11 + H, LSH = UB + SB;
  __device__ static __forceinline__ uint32_t wmake(int u, int src, int len) {
    return (uint32_t)u | ((uint32_t)src << UB) | ((uint32_t)len << LSH);
  }
  __device__ static __forceinline__ int wunit(uint32_t w) { return (int)(w & ((1u << UB) - 1u)); }
  __device__ static __forceinline__ int wsrc(uint32_t w) { return (int)((w >> UB) & ((1u << SB) - 1u)); }
  __device__ static __forceinline__ int wlen(uint32_t w) { return (int)(w >> LSH); }
};
constexpr uint32_t BF = 0xFFu, BX = 0xFDu, BS = 0xF8u;  // filler, expansion, special k = BS+k

// class byte per input byte value
enum : uint32_t { C_W = 1, C_I = 2, C_S = 4, C_D = 8, C_UP = 16, C_X = 32, C_CS = 64 };

template <int H>
struct WaveLds {
  using G = Geo<H>;
  // raw bytes (step 1); afterwards the same bytes hold the pieces: uid[u] =
  // the id of a unit done with one piece (specials, [UNK], first-probe hits),
  // upo[u] = offset of a WordPiece unit's pieces in mp (bump-allocated, <=
  // its byte length each), 0xFFFF = uid
  union {
    uint32_t rp[G::CAP / 4 + 4];
    struct {
      uint16_t uid[G::UCAP];
      uint16_t upo[G::UCAP];
      uint16_t mp[G::MPCAP];
    } pcs;
  };
  uint32_t nb[G::NBUF / 4];     // normalised bytes in window coordinates; side buffer at [CAP, CAP+DCAP)
  uint32_t brk[64 * H];          // break bits: unit starts, spaces, sentence starts
  uint32_t dm[64 * H];           // dirty bits: filler / expansion marker bytes
  uint32_t sb[64 * H];           // sentence-start bits
  uint32_t urec[G::UCAP];       // window position | sentence << 16
  uint32_t uwp[G::UCAP];        // WordPiece entry (Geo::wmake; 0: none), then the work list in place
  uint8_t ucnt[G::UCAP];        // pieces per unit
  uint16_t sst[G::NSCAP + 2];   // sentence starts (window coordinates)
  uint16_t stot[G::NSCAP];      // tokens per sentence
  uint32_t xent[G::XCAP];       // table entry of each expansion marker
  uint8_t xlen[G::XCAP];        // its normalised byte length
  int32_t misc[4];           // 0 side-buffer cursor, 1 #markers, 2 overflow, 3 mp cursor
};

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <int H>
__device__ __forceinline__ uint32_t rawb(const WaveLds<H>& L, int p) { return reinterpret_cast<const uint8_t*>(L.rp)[p]; }
template <int H>
__device__ __forceinline__ uint32_t nbyte(const WaveLds<H>& L, int p) { return reinterpret_cast<const uint8_t*>(L.nb)[p]; }
template <int H>
__device__ __forceinline__ void nput(WaveLds<H>& L, int p, uint32_t v) { reinterpret_cast<uint8_t*>(L.nb)[p] = (uint8_t)v; }

// bit q of each byte of c -> 4 bits (byte 0 -> bit 0)
__device__ __forceinline__ uint32_t gather4(uint32_t c, int q) { return (((c >> q) & 0x01010101u) * 0x01020408u) >> 24; }

__device__ __forceinline__ int64_t uni64(int64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int lane_rank(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t wave_excl(uint32_t v, int lane, uint32_t* total) {
  (void)lane;
  const uint32_t x = wave_incl_add(v);
  *total = lane_get(x, 63);
  return x - v;
}

template <int H>
__device__ __forceinline__ int utf8_put(WaveLds<H>& L, int p, uint32_t c) {
  if (c < 0x80) { nput(L, p, c); return 1; }
  if (c < 0x800) { nput(L, p, 0xC0 | (c >> 6)); nput(L, p + 1, 0x80 | (c & 0x3F)); return 2; }
  if (c < 0x10000) {
    nput(L, p, 0xE0 | (c >> 12)); nput(L, p + 1, 0x80 | ((c >> 6) & 0x3F)); nput(L, p + 2, 0x80 | (c & 0x3F));
    return 3;
  }
  nput(L, p, 0xF0 | (c >> 18)); nput(L, p + 1, 0x80 | ((c >> 12) & 0x3F));
  nput(L, p + 2, 0x80 | ((c >> 6) & 0x3F)); nput(L, p + 3, 0x80 | (c & 0x3F));
  return 4;
}

// first break position > p (a unit's span end), at most nb
template <int H>
__device__ __forceinline__ int span_end(const WaveLds<H>& L, int p, int nb) {
  int w = p >> 5;
  uint32_t m = L.brk[w] & ~((2u << (p & 31)) - 1u);
  while (m == 0) {
    ++w;
    if ((w << 5) >= nb) return nb;
    m = L.brk[w];
  }
  return min((w << 5) + __ffs(m) - 1, nb);
}

template <int H>
__device__ __forceinline__ bool span_dirty(const WaveLds<H>& L, int p, int q) {
  for (int w = p >> 5; (w << 5) < q; ++w) {
    const int lo = max(p - (w << 5), 0), hi = min(q - (w << 5), 32);
    const uint32_t m = (hi >= 32 ? ~0u : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
    if (L.dm[w] & m) return true;
  }
  return false;
}

// Compact / expand the dirty span [p, q) into the side buffer.  Returns its
// normalised length (source in *src), -1 on overflow (flagged in misc[2]).
template <int H>
__device__ int dirty_normalize(WaveLds<H>& L, const TokParams& P, int p, int q, int* src) {
  int len = 0;
  for (int i = p; i < q;) {
    const uint32_t b = nbyte(L, i);
    if (b == BF) {
      ++i;
    } else if (b == BX) {
      len += L.xlen[nbyte(L, i + 1)];
      i += 2;
    } else {
      ++len;
      ++i;
    }
  }
  if (len == 0) return 0;
  const int off = atomicAdd(&L.misc[0], len);
  if (off + len > Geo<H>::DCAP) {
    L.misc[2] = 1;
    return -1;
  }
  int o = Geo<H>::CAP + off;
  *src = o;
  for (int i = p; i < q;) {
    const uint32_t b = nbyte(L, i);
    if (b == BF) {
      ++i;
    } else if (b == BX) {
      const uint32_t e = L.xent[nbyte(L, i + 1)];
      if (ent_kind(e) == KIND_MULTI) {
        const uint4 m = P.multi[ent_payload(e)];
        o += utf8_put(L, o, ent_payload(m.y));
        o += utf8_put(L, o, ent_payload(m.z));
        if (m.x > 2) o += utf8_put(L, o, ent_payload(m.w));
      } else {
        o += utf8_put(L, o, ent_payload(e));
      }
      i += 2;
    } else {
      nput(L, o++, b);
      ++i;
    }
  }
  return len;
}

template <int H>
__device__ __forceinline__ int count_chars(const WaveLds<H>& L, int src, int len) {
  int n = 0;
  for (int i = 0; i < len; ++i) n += (nbyte(L, src + i) & 0xC0u) != 0x80u;
  return n;
}

// bytes [24, len) of a candidate against the vocab pool
template <int H>
__device__ __forceinline__ bool long_eq(const WaveLds<H>& L, const TokParams& P, int s, int len, uint32_t off) {
  for (int k = 24; k < len; ++k)
    if (nbyte(L, s + k) != P.pool[off + k]) return false;
  return true;
}


// the first min(len, 24) bytes at s as six little-endian dwords, zero beyond
struct Key6 {
  uint32_t d0, d1, d2, d3, d4, d5;
};
template <int H>
__device__ __forceinline__ Key6 load_key(const WaveLds<H>& L, int s, int len) {
  const int a = s >> 2;
  const uint32_t sh = (uint32_t)(s & 3);
  const uint32_t x0 = L.nb[a], x1 = L.nb[a + 1], x2 = L.nb[a + 2], x3 = L.nb[a + 3], x4 = L.nb[a + 4],
                 x5 = L.nb[a + 5], x6 = L.nb[a + 6];
  const int lc = min(len, 24);
  auto m = [&](int i, uint32_t c) {
    const int rem = lc - 4 * i;
    return rem >= 4 ? c : rem <= 0 ? 0u : (c & ((1u << (8 * rem)) - 1u));
  };
  Key6 k;
  k.d0 = m(0, __builtin_amdgcn_alignbyte(x1, x0, sh));
  k.d1 = m(1, __builtin_amdgcn_alignbyte(x2, x1, sh));
  k.d2 = m(2, __builtin_amdgcn_alignbyte(x3, x2, sh));
  k.d3 = m(3, __builtin_amdgcn_alignbyte(x4, x3, sh));
  k.d4 = m(4, __builtin_amdgcn_alignbyte(x5, x4, sh));
  k.d5 = m(5, __builtin_amdgcn_alignbyte(x6, x5, sh));
  return k;
}
// == vhash (common.h) of a loaded key; *bk = its Bloom key (vbkey)
__device__ __forceinline__ uint32_t key_hash(const Key6& k, int len, uint32_t cont, uint32_t* bk) {
  const int lc = min(len, 24);
  uint32_t h = VSEED, hq = VSEED, tail = 0;
#define TOK4_KH(i, di)            \
  if (lc > 4 * (i)) {             \
    if (lc < 4 * (i) + 4) {       \
      hq = h;                     \
      tail = di;                  \
    }                             \
    h = vmix(h, di);              \
  }
  TOK4_KH(0, k.d0)
  TOK4_KH(1, k.d1)
  TOK4_KH(2, k.d2)
  TOK4_KH(3, k.d3)
  TOK4_KH(4, k.d4)
  TOK4_KH(5, k.d5)
#undef TOK4_KH
  if ((lc & 3) == 0) hq = h;
  *bk = vbkey(hq, tail, (uint32_t)len, cont);
  return vfinal(h, (uint32_t)len, cont);
}
// branch-free (an && chain lets the compiler sink the slot's other loads
// behind the first compare: a second dependent round trip on every hit)
__device__ __forceinline__ bool slot_eq(const uint4& a, const uint4& b, const Key6& k, uint32_t want) {
  return (((b.z & 0xFFFF0000u) ^ want) | (a.x ^ k.d0) | (a.y ^ k.d1) | (a.z ^ k.d2) | (a.w ^ k.d3) | (b.x ^ k.d4) |
          (b.y ^ k.d5)) == 0u;
}

template <int WAVES, bool BLOOM, bool DBG, int H>
__global__ __launch_bounds__(64 * WAVES) void tok4_kernel(TokParams P, const int64_t* tile_sent, int64_t n_tiles,
                                                          int32_t* fb_list, int32_t* fb_count) {
  using G = Geo<H>;
  constexpr int CAP = G::CAP, UCAP = G::UCAP, NSCAP = G::NSCAP, XCAP = G::XCAP, MPCAP = G::MPCAP;
  __shared__ WaveLds<H> Ls[WAVES];
  __shared__ uint32_t ctab32[64];
  __shared__ uint32_t bloom[BLOOM ? BLOOM_WORDS : 1];
  // ---- prologue: class table (from the unicode table's ASCII page), Bloom --
  if (threadIdx.x < 64) {
    uint32_t word = 0;
    for (int k = 0; k < 4; ++k) {
      const uint32_t b = threadIdx.x * 4 + k;
      uint32_t c;
      if (b < 128) {
        const uint32_t e = P.pages[(uint32_t)P.top[0] * 256u + b];
        const uint32_t kind = ent_kind(e), cls = ent_cls(e);
        c = C_CS;
        if (kind == KIND_DROP_T || kind == KIND_DROP_D) c |= C_W | C_D;
        else if (cls == CLS_SPACE) c |= C_S;
        else if (cls == CLS_ISOLATE) c |= C_I;
        else c |= C_W;
        if (kind == KIND_MAP && cls == CLS_OTHER) c |= C_UP;  // A-Z -> a-z (checked at lddl_create)
        if (b == '[') c |= C_X;
      } else {
        c = b >= 0xC0 ? (C_X | C_CS) : 0u;
      }
      word |= c << (8 * k);
    }
    ctab32[threadIdx.x] = word;
  }
  if (BLOOM)
    for (int i = threadIdx.x; i < BLOOM_WORDS; i += 64 * WAVES) bloom[i] = P.vbloom[i];
  __syncthreads();
  const uint8_t* ctab = reinterpret_cast<const uint8_t*>(ctab32);
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  WaveLds<H>& L = Ls[wv];
  const int64_t base = P.sent_off[0];
  const int64_t nwaves = (int64_t)gridDim.x * WAVES;
  const int64_t n_work = (n_tiles + H - 1) / H;  // a wave's tile = H consecutive 1 KiB tiles
  constexpr bool dbg = DBG;
  uint64_t acc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tprev = 0;
#define STAMP(k)                                      \
  if (dbg) {                                          \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    acc[k] += t_ - tprev;                             \
    tprev = t_;                                       \
  }
  for (int64_t t = (int64_t)blockIdx.x * WAVES + wv; t < n_work; t += nwaves) {
    wsync();
    if (dbg) tprev = __builtin_amdgcn_s_memtime();
    const int64_t t0 = t * H, t1 = min(t0 + H, n_tiles);
    // the fallback kernel re-runs listed 1 KiB tiles
    auto fallback = [&]() {
      if (lane == 0) {
        const int at = atomicAdd(fb_count, (int)(t1 - t0));
        for (int64_t q = t0; q < t1; ++q) fb_list[at + (q - t0)] = (int32_t)q;
      }
    };
    const int64_t sa = uni64(tile_sent[t0]), sb = uni64(tile_sent[t1]);
    if (sa >= sb) continue;
    const int64_t A = uni64(P.sent_off[sa]), B = uni64(P.sent_off[sb]);
    const int aoff = (int)(reinterpret_cast<uintptr_t>(P.bytes + A) & 15u);
    const uint8_t* wbase = P.bytes + (A - aoff);  // 16-B aligned (derived from the global pointer: global loads)
    const int64_t nb64 = (B - A) + aoff;
    const int ns = (int)(sb - sa);
    if (dbg) acc[10] += 1;
    if (nb64 > CAP || ns > NSCAP) {
      fallback();
      if (dbg) acc[11] += 1;
      continue;
    }
    const int nb = (int)nb64;
    // ---- sentence starts ----------------------------------------------------
#pragma unroll
    for (int h = 0; h < H; ++h) L.sb[h * 64 + lane] = 0;
    if (lane == 0) {
      L.misc[0] = 0;
      L.misc[1] = 0;
      L.misc[2] = 0;
    }
    for (int j = lane; j < ns; j += 64) L.stot[j] = 0;
    wsync();
    for (int j = lane; j < ns; j += 64) {
      const int pos = (int)(P.sent_off[sa + j] - A) + aoff;
      L.sst[j] = (uint16_t)pos;
      if (pos < nb) atomicOr(&L.sb[pos >> 5], 1u << (pos & 31));
    }
    // ---- 1: raw bytes -> masks + normalised bytes in place ------------------
    // half h covers window bytes [2048 h, 2048 (h + 1)), lane l its 32 bytes
    // from 2048 h + 32 l; masks per half in registers (constant indices)
    uint32_t W[H], I[H], S[H], CS[H], D[H], X[H], inwin[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const int p0 = h * 2048 + lane * 32;
      uint4 v0 = make_uint4(0, 0, 0, 0), v1 = v0;
      {
        // 16-B aligned blocks holding >= 1 window byte: never past a page
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4* gp = reinterpret_cast<const u32x4*>(wbase) + 2 * (h * 64 + lane);
        if (p0 < nb) {  // streamed once: non-temporal, keep L2 for the vocab table
          const u32x4 a = __builtin_nontemporal_load(gp);
          v0 = make_uint4(a.x, a.y, a.z, a.w);
        }
        if (p0 + 16 < nb) {
          const u32x4 a = __builtin_nontemporal_load(gp + 1);
          v1 = make_uint4(a.x, a.y, a.z, a.w);
        }
      }
      *reinterpret_cast<uint4*>(&L.rp[(h * 64 + lane) * 8]) = v0;
      *reinterpret_cast<uint4*>(&L.rp[(h * 64 + lane) * 8 + 4]) = v1;
      const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      uint32_t Wh = 0, Ih = 0, Sh = 0, CSh = 0, Dh = 0, Xh = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t x = w[k];
        const uint32_t c = (uint32_t)ctab[x & 0xFFu] | ((uint32_t)ctab[(x >> 8) & 0xFFu] << 8) |
                           ((uint32_t)ctab[(x >> 16) & 0xFFu] << 16) | ((uint32_t)ctab[x >> 24] << 24);
        L.nb[(h * 64 + lane) * 8 + k] = (x + ((c & 0x10101010u) << 1)) | (((c >> 3) & 0x01010101u) * 0xFFu);
        const int sh = 4 * k;
        Wh |= gather4(c, 0) << sh;
        Ih |= gather4(c, 1) << sh;
        Sh |= gather4(c, 2) << sh;
        Dh |= gather4(c, 3) << sh;
        Xh |= gather4(c, 5) << sh;
        CSh |= gather4(c, 6) << sh;
      }
      const int wlo = min(max(aoff - p0, 0), 32), whi = min(max(nb - p0, 0), 32);
      inwin[h] = (whi >= 32 ? ~0u : ((1u << whi) - 1u)) & (wlo >= 32 ? 0u : ~((1u << wlo) - 1u));
      W[h] = Wh; I[h] = Ih; S[h] = Sh; CS[h] = CSh; D[h] = Dh; X[h] = Xh & inwin[h];
    }
    wsync();
    STAMP(0);
    bool bad = false;
    uint32_t spm[H], spw[H], spd[H];  // per half: this lane's last char / special running into the next lane
#pragma unroll
    for (int h = 0; h < H; ++h) {
    const int p0 = h * 2048 + lane * 32;
    uint32_t sp_m = 0, sp_w = 0, sp_d = 0;
    uint32_t Wh = W[h], Ih = I[h], Sh = S[h], CSh = CS[h], Dh = D[h];
    for (uint32_t xm = X[h]; xm;) {
      const int i = __ffs(xm) - 1;
      xm &= xm - 1;
      const int p = p0 + i;
      const uint32_t b = rawb(L, p);
      if (b == '[') {
        int se = nb;  // end of p's sentence
        for (int j = 1; j < ns; ++j)
          if (L.sst[j] > p) { se = L.sst[j]; break; }
        int len = 0, sk = -1;
        if (p + 5 <= se) {
          const uint32_t c1 = rawb(L, p + 1), c2 = rawb(L, p + 2), c3 = rawb(L, p + 3), c4 = rawb(L, p + 4);
          if (c1 == 'P' && c2 == 'A' && c3 == 'D' && c4 == ']') { sk = 0; len = 5; }
          else if (c1 == 'U' && c2 == 'N' && c3 == 'K' && c4 == ']') { sk = 1; len = 5; }
          else if (c1 == 'C' && c2 == 'L' && c3 == 'S' && c4 == ']') { sk = 2; len = 5; }
          else if (c1 == 'S' && c2 == 'E' && c3 == 'P' && c4 == ']') { sk = 3; len = 5; }
          else if (c1 == 'M' && c2 == 'A' && c3 == 'S' && c4 == 'K' && p + 6 <= se && rawb(L, p + 5) == ']') { sk = 4; len = 6; }
        }
        if (sk >= 0) {
          nput(L, p, BS + (uint32_t)sk);
          const uint64_t cov = ((1ull << (len - 1)) - 1ull) << (i + 1);
          const uint32_t cl = (uint32_t)cov;
          Wh &= ~cl;
          Ih &= ~cl;
          Sh &= ~cl;
          CSh &= ~cl;
          Dh &= ~cl;
          sp_m |= (uint32_t)(cov >> 32);
        }
      } else {
        const int n = utf8_len(b);
        uint32_t cp = b & (0x3Fu >> (n - 1));
        for (int q = 1; q < n; ++q) cp = (cp << 6) | (rawb(L, p + q) & 0x3Fu);
        if (cp > 0x10FFFF) cp = 0xFFFD;
        const uint32_t e = table_entry(P, cp);
        const uint32_t kind = ent_kind(e), cls = ent_cls(e);
        const uint64_t span = ((1ull << n) - 1ull) << i;
        bool dirty = false, wordc = false;
        if (ent_rank(e) != 0) bad = true;
        if (kind == KIND_DROP_T || kind == KIND_DROP_D) {
          for (int q = 0; q < n; ++q) nput(L, p + q, BF);
          dirty = true;
          wordc = true;
        } else if (cls == CLS_SPACE) {
          Sh |= 1u << i;
        } else {
          if (cls == CLS_ISOLATE) Ih |= 1u << i;
          else wordc = true;
          if (kind != KIND_IDENT) {
            uint32_t c0 = ent_payload(e), c1 = 0, c2 = 0;
            int nc = 1;
            if (kind == KIND_MULTI) {
              const uint4 m = P.multi[ent_payload(e)];
              nc = (int)m.x;
              c0 = ent_payload(m.y);
              c1 = ent_payload(m.z);
              c2 = ent_payload(m.w);
              if ((ent_rank(m.y) | ent_rank(m.z) | (nc > 2 ? ent_rank(m.w) : 0u)) != 0) bad = true;
            }
            const int T = utf8_enc_len(c0) + (nc > 1 ? utf8_enc_len(c1) : 0) + (nc > 2 ? utf8_enc_len(c2) : 0);
            if (T <= n) {
              int o = p + utf8_put(L, p, c0);
              if (nc > 1) o += utf8_put(L, o, c1);
              if (nc > 2) o += utf8_put(L, o, c2);
              for (; o < p + n; ++o) nput(L, o, BF);
              dirty = T < n;
            } else {
              const int xi = atomicAdd(&L.misc[1], 1);
              if (xi >= XCAP) {
                bad = true;
              } else {
                L.xent[xi] = e;
                L.xlen[xi] = (uint8_t)T;
                nput(L, p, BX);
                nput(L, p + 1, (uint32_t)xi);
                for (int q = 2; q < n; ++q) nput(L, p + q, BF);
              }
              dirty = true;
            }
          }
        }
        const uint32_t slo = (uint32_t)span, shi = (uint32_t)(span >> 32);
        if (wordc) {
          Wh |= slo;
          sp_w |= shi;
        }
        if (dirty) {
          Dh |= slo;
          sp_d |= shi;
        }
        sp_m |= shi;
      }
    }
    W[h] = Wh; I[h] = Ih; S[h] = Sh; CS[h] = CSh; D[h] = Dh;
    spm[h] = sp_m; spw[h] = sp_w; spd[h] = sp_d;
    }  // halves
#pragma unroll
    for (int h = 0; h < H; ++h) {
      // carry into lane 0 of half h > 0 from lane 63 of half h - 1
      uint32_t im = wave_shr1(spm[h]), iw = wave_shr1(spw[h]), id = wave_shr1(spd[h]);  // lane 0: 0
      if (h > 0) {
        const uint32_t pm = lane_get(spm[h > 0 ? h - 1 : 0], 63), pw_ = lane_get(spw[h > 0 ? h - 1 : 0], 63),
                       pd = lane_get(spd[h > 0 ? h - 1 : 0], 63);
        if (lane == 0) {
          im = pm;
          iw = pw_;
          id = pd;
        }
      }
      W[h] = ((W[h] & ~im) | iw) & inwin[h];
      I[h] &= ~im & inwin[h];
      S[h] &= ~im & inwin[h];
      CS[h] &= ~im & inwin[h];
      D[h] = ((D[h] & ~im) | id) & inwin[h];
    }
    const bool wbad = __any(bad);
    wsync();
    STAMP(1);
    // ---- 2: units -----------------------------------------------------------
    uint32_t U[H], SBm[H];
    int ub[H], sbb[H];
    int n = 0, nstarts = 0;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const uint32_t SBh = L.sb[h * 64 + lane];
      uint32_t carry = wave_shr1(W[h]) >> 31;
      if (h > 0) {
        const uint32_t pc = lane_get(W[h > 0 ? h - 1 : 0], 63) >> 31;
        if (lane == 0) carry = pc;
      }
      const uint32_t pw = (W[h] << 1) | ((lane || h) ? carry : 0u);
      const uint32_t Uh = CS[h] & (I[h] | (W[h] & (~pw | SBh)));
      L.brk[h * 64 + lane] = Uh | (S[h] & CS[h]) | SBh;
      L.dm[h * 64 + lane] = D[h];
      uint32_t tot;
      // one scan for both: units (low 16 bits) and sentence starts (high)
      const uint32_t ex = wave_excl((uint32_t)__popc(Uh) | ((uint32_t)__popc(SBh) << 16), lane, &tot);
      ub[h] = n + (int)(ex & 0xFFFFu);
      sbb[h] = nstarts + (int)(ex >> 16);
      n += (int)(tot & 0xFFFFu);
      nstarts += (int)(tot >> 16);
      U[h] = Uh;
      SBm[h] = SBh;
    }
    // every sentence start distinct (no empty sentence shares one): a unit's
    // sentence is the number of starts at or before it, minus one
    const bool starts_distinct = nstarts == ns;
    if (wbad) {
      fallback();
      if (dbg) acc[11] += 1;
      continue;
    }
    // units are processed in rounds of UCAP; a sentence running across two
    // rounds continues its token count (stot) in the next one
    int prev_sent = -1;
    for (int rb = 0; rb < n; rb += UCAP) {
      const int nr = min(UCAP, n - rb);
      if (lane == 0) {
        L.misc[0] = 0;
        L.misc[3] = 0;
      }
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const int p0 = h * 2048 + lane * 32;
        int u = ub[h];
        for (uint32_t m = U[h]; m; m &= m - 1, ++u) {
          if (u < rb || u >= rb + nr) continue;
          const int b = __ffs(m) - 1, p = p0 + b;
          int lo;
          if (starts_distinct) {
            lo = sbb[h] + __popc(SBm[h] & ((2u << b) - 1u)) - 1;
          } else {
            lo = 0;  // last sentence starting at or before p
            int hi = ns - 1;
            while (lo < hi) {
              const int mid = (lo + hi + 1) >> 1;
              if ((int)L.sst[mid] <= p) lo = mid;
              else hi = mid - 1;
            }
          }
          L.urec[u - rb] = (uint32_t)p | ((uint32_t)lo << 16);
        }
      }
      wsync();
      STAMP(2);
    // ---- 3: prep (spans, dirty words, specials, long words) -----------------
    int nwl = 0;
    for (int r = 0; r < nr; r += 64) {
      const int u = r + lane;
      bool need = false;
      if (u < nr) {
        const int p = (int)(L.urec[u] & 0xFFFFu);
        const uint32_t b0 = nbyte(L, p);
        int cnt = -1;
        if (b0 >= BS && b0 < BS + 5) {
          L.pcs.uid[u] = (uint16_t)P.special[b0 - BS];
          cnt = 1;
        } else {
          const int q = span_end(L, p, nb);
          int src = p, len = q - p;
          if (span_dirty(L, p, q)) len = max(dirty_normalize(L, P, p, q, &src), 0);
          if (len == 0) {
            cnt = 0;
          } else if (len > 100 && count_chars(L, src, len) > 100) {
            L.pcs.uid[u] = (uint16_t)P.unk;
            cnt = 1;
          } else {
            need = true;
            L.uwp[u] = G::wmake(u, src, len);
          }
        }
        if (cnt >= 0) L.ucnt[u] = (uint8_t)cnt;
        L.pcs.upo[u] = 0xFFFFu;
        if (!need) L.uwp[u] = 0;
      }
      const uint64_t bm = __ballot(need);
      nwl += __popcll(bm);
    }
    wsync();
    // ---- 3b: first probe of every pending unit (its whole word, the common
    //      hit) with 4 bucket loads in flight per lane; hits leave the queue
    {
      const int mb0 = (int)P.maxb[0];
      const uint32_t vmask = P.vt_mask;
      auto bl_ok = [&](uint32_t h) {
        if (!BLOOM) return true;
        const uint32_t bb = vbloom_bits(h);
        return (bloom[vbloom_word(h)] & bb) == bb;
      };
#define TOK4_FP_ISSUE(k)                                                       \
  uint4 fa##k = make_uint4(0, 0, 0, 0), fb##k = fa##k;                         \
  bool fact##k = false;                                                        \
  {                                                                            \
    const int u = (k) * 64 + lane;                                             \
    const uint32_t w = u < nr ? L.uwp[u] : 0u;                                 \
    const int len = G::wlen(w);                                                \
    if (w != 0 && len <= 24 && len <= mb0) {                                   \
      uint32_t bk;                                                             \
      const uint32_t h = key_hash(load_key(L, G::wsrc(w), len), len, 0u, &bk); \
      if (bl_ok(bk)) {                                                         \
        const uint4* bk = P.vt + 4 * (h & vmask);                              \
        fa##k = bk[0];                                                         \
        fb##k = bk[1];                                                         \
        fact##k = true;                                                        \
      }                                                                        \
    }                                                                          \
  }
#define TOK4_FP_CHECK(k)                                                       \
  if (fact##k) {                                                               \
    const int u = (k) * 64 + lane;                                             \
    const uint32_t w = L.uwp[u];                                               \
    const int len = G::wlen(w);                                                \
    const Key6 key = load_key(L, G::wsrc(w), len);                             \
    if (slot_eq(fa##k, fb##k, key, ((uint32_t)len << 16) | 0x80000000u)) {      \
      L.pcs.uid[u] = (uint16_t)(fb##k.z & 0xFFFFu);                            \
      L.ucnt[u] = 1;                                                           \
      L.uwp[u] = 0;                                                            \
      if (dbg) acc[6] += 1;                                                    \
    }                                                                          \
  }
      {
        TOK4_FP_ISSUE(0)
        TOK4_FP_ISSUE(1)
        TOK4_FP_ISSUE(2)
        TOK4_FP_ISSUE(3)
        TOK4_FP_CHECK(0)
        TOK4_FP_CHECK(1)
        TOK4_FP_CHECK(2)
        TOK4_FP_CHECK(3)
      }
      if constexpr (H == 2) {  // units 256..511: a second batch of 4 per lane
        TOK4_FP_ISSUE(4)
        TOK4_FP_ISSUE(5)
        TOK4_FP_ISSUE(6)
        TOK4_FP_ISSUE(7)
        TOK4_FP_CHECK(4)
        TOK4_FP_CHECK(5)
        TOK4_FP_CHECK(6)
        TOK4_FP_CHECK(7)
      }
#undef TOK4_FP_ISSUE
#undef TOK4_FP_CHECK
      static_assert(UCAP == 256 * H && H <= 2, "first-probe batches are unrolled for 4 units per lane");
    }
    wsync();
    // work list (in place over uwp), longest first: long words are the OOV
    // ones needing many probes, and starting them first keeps the tail short
    {
      constexpr int K = UCAP / 64;
      uint32_t ent[K];
#pragma unroll
      for (int k = 0; k < K; ++k) ent[k] = k * 64 + lane < nr ? L.uwp[k * 64 + lane] : 0u;
      wsync();
      int at = 0;
#pragma unroll
      for (int pass = 0; pass < 2; ++pass)
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const bool take = ent[k] != 0 && (G::wlen(ent[k]) >= 10) == (pass == 0);
          const uint64_t bm = __ballot(take);
          if (take) L.uwp[at + lane_rank(bm)] = ent[k];
          at += __popcll(bm);
        }
      nwl = at;  // first-probe hits have left the queue
    }
    wsync();
    if (P.dbg_mode == 1) {  // ablation (LDDL_TOK_ABLATE=1, diagnostics only): no WordPiece loop
      for (int i = lane; i < nwl; i += 64) {
        const int u = G::wunit(L.uwp[i]);
        L.pcs.uid[u] = (uint16_t)P.unk;
        L.ucnt[u] = 1;
      }
      nwl = 0;
      wsync();
    }
    if (L.misc[2]) break;  // side buffer overflow: the whole tile falls back
    STAMP(3);
    if (dbg) acc[8] += nr;
    // ---- 4: WordPiece on the work queue --------------------------------------
    {
      const int mb0 = (int)P.maxb[0], mb1 = (int)P.maxb[1];
      const uint32_t vmask = P.vt_mask;
      int u = -1, s = 0, we = 0, e = 0, pb = 0, np = 0, slot = -1;
      uint32_t cont = 0, hcur = 0;
      bool asc = false;
      // candidate bytes [s, s+24) as dwords c0..c5 and the prefix mixes
      // H0..H6 (H(k+1) = vmix(Hk, ck)): named scalars, never an indexed
      // array, so nothing is demoted to scratch by dynamic indexing
      uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0;
      uint32_t H0 = VSEED, H1 = 0, H2 = 0, H3 = 0, H4 = 0, H5 = 0, H6 = 0;
      auto load_cand = [&]() {
        const int a = s >> 2;
        const uint32_t sh = (uint32_t)(s & 3);
        const uint32_t x0 = L.nb[a], x1 = L.nb[a + 1], x2 = L.nb[a + 2], x3 = L.nb[a + 3], x4 = L.nb[a + 4],
                       x5 = L.nb[a + 5], x6 = L.nb[a + 6];
        c0 = __builtin_amdgcn_alignbyte(x1, x0, sh);
        c1 = __builtin_amdgcn_alignbyte(x2, x1, sh);
        c2 = __builtin_amdgcn_alignbyte(x3, x2, sh);
        c3 = __builtin_amdgcn_alignbyte(x4, x3, sh);
        c4 = __builtin_amdgcn_alignbyte(x5, x4, sh);
        c5 = __builtin_amdgcn_alignbyte(x6, x5, sh);
        H1 = vmix(H0, c0);
        H2 = vmix(H1, c1);
        H3 = vmix(H2, c2);
        H4 = vmix(H3, c3);
        H5 = vmix(H4, c4);
        H6 = vmix(H5, c5);
        asc = ((c0 | c1 | c2 | c3 | c4 | c5) & 0x80808080u) == 0;
      };
      auto selH = [&](int q) {
        return q <= 0 ? H0 : q == 1 ? H1 : q == 2 ? H2 : q == 3 ? H3 : q == 4 ? H4 : q == 5 ? H5 : H6;
      };
      auto selD = [&](int q) {
        return q <= 0 ? c0 : q == 1 ? c1 : q == 2 ? c2 : q == 3 ? c3 : q == 4 ? c4 : c5;
      };
      auto hash_len = [&](int l) {  // == vhash of the candidate [s, s+l)
        const int lc = min(l, 24), q = lc >> 2, r = lc & 3;
        uint32_t h = selH(q);
        if (r) h = vmix(h, selD(q) & ((1u << (8 * r)) - 1u));
        return vfinal(h, (uint32_t)l, cont);
      };
      auto bkey_len = [&](int l) {  // == vbkey of the candidate [s, s+l)
        const int lc = min(l, 24), q = lc >> 2, r = lc & 3;
        return vbkey(selH(q), r ? selD(q) & ((1u << (8 * r)) - 1u) : 0u, (uint32_t)l, cont);
      };
      auto bloom_ok = [&](uint32_t h) {
        if (!BLOOM) return true;
        const uint32_t bb = vbloom_bits(h);
        return (bloom[vbloom_word(h)] & bb) == bb;
      };
      auto shrink = [&]() {  // previous char boundary
        --e;
        if (!(asc && e - s < 24))
          while (e > s && (nbyte(L, e) & 0xC0u) == 0x80u) --e;
      };
      auto start_piece = [&](int maxb) {
        slot = -1;
        load_cand();
        e = min(we, s + maxb);
        if (e < we && !(asc && e - s < 24))
          while (e > s && (nbyte(L, e) & 0xC0u) == 0x80u) --e;
      };
      // pieces: the first 8 in registers (u16 pairs), allocated exactly in mp
      // when the word ends; a word reaching 8 pieces spills to a block of its
      // byte length (#pieces <= #bytes)
      uint32_t pr0 = 0, pr1 = 0, pr2 = 0, pr3 = 0;
      int ulen = 0;
      auto mp_alloc = [&](int n) {
        const int at = atomicAdd(&L.misc[3], n);
        if (at + n > MPCAP) {  // piece buffer exhausted: the tile falls back
          L.misc[2] = 1;
          return -1;
        }
        return at;
      };
      auto reg_piece = [&](int q) {
        const uint32_t w = q < 2 ? pr0 : q < 4 ? pr1 : q < 6 ? pr2 : pr3;
        return (uint16_t)(w >> ((q & 1) * 16));
      };
      auto put_piece = [&](uint32_t id) {
        if (pb >= 0) {
          L.pcs.mp[pb + np] = (uint16_t)id;
        } else if (np < 8) {
          const uint32_t sh = (uint32_t)(np & 1) * 16u, keep = ~(0xFFFFu << sh), v = id << sh;
          const int w = np >> 1;
          pr0 = w == 0 ? (pr0 & keep) | v : pr0;
          pr1 = w == 1 ? (pr1 & keep) | v : pr1;
          pr2 = w == 2 ? (pr2 & keep) | v : pr2;
          pr3 = w == 3 ? (pr3 & keep) | v : pr3;
        } else {
          pb = mp_alloc(ulen);
          if (pb >= 0) {
            for (int q = 0; q < 8; ++q) L.pcs.mp[pb + q] = reg_piece(q);
            L.pcs.mp[pb + 8] = (uint16_t)id;
          }
        }
        ++np;
      };
      auto finish = [&]() {  // the word's pieces are complete
        if (pb < 0 && np <= 8) {
          pb = mp_alloc(np);
          if (pb >= 0)
            for (int q = 0; q < np; ++q) L.pcs.mp[pb + q] = reg_piece(q);
        }
        L.pcs.upo[u] = (uint16_t)(pb >= 0 ? pb : 0);
        L.ucnt[u] = (uint8_t)(pb >= 0 ? np : 0);
        u = -1;
      };
      auto begin = [&](uint32_t w) {
        u = G::wunit(w);
        s = G::wsrc(w);
        ulen = G::wlen(w);
        we = s + ulen;
        pb = -1;
        np = 0;
        cont = 0;
        start_piece(mb0);
      };
      if (lane < nwl) begin(L.uwp[lane]);
      int next = 64;
      for (;;) {
        if (__ballot(u >= 0) == 0 && next >= nwl) break;
        if (dbg) acc[9] += 1;
        STAMP(4);
        if (u >= 0) {
          bool fail = false;
          if (slot < 0) {
            // longest candidate <= e - s the Bloom filter does not rule out
            int len = e - s;
            bool found = false;
            if (asc && len <= 24) {
              // ASCII: every length is a char boundary.  Dword group k holds
              // lengths 4k+1..4k+4, hashed from Hk / H(k+1) with constant
              // register indices; groups from the top down.
              int fl = 0;
              // highest reachable group: k+1 only if some vocab key longer
              // than 4(k+1) bytes starts with the candidate's first 4(k+1)
              // (branch-free: the Bloom words are always in range)
              int ga = 0;
#define TOK4_EXT(j, Hj1) \
  ga = ((ga == (j)) & (4 * ((j) + 1) < len) & bloom_ok(vbkey_ext(Hj1, 4 * ((j) + 1), cont))) ? (j) + 1 : ga;
              TOK4_EXT(0, H1)
              TOK4_EXT(1, H2)
              TOK4_EXT(2, H3)
              TOK4_EXT(3, H4)
              TOK4_EXT(4, H5)
#undef TOK4_EXT
#define TOK4_GROUP(k, Hk, Hk1, ck)                                                                  \
  if (fl == 0 && 4 * (k) < len && (k) <= ga) {                                                      \
    const uint32_t g4 = vbkey(Hk1, 0u, 4 * (k) + 4, cont), g3 = vbkey(Hk, (ck) & 0xFFFFFFu, 4 * (k) + 3, cont), \
                   g2 = vbkey(Hk, (ck) & 0xFFFFu, 4 * (k) + 2, cont),                               \
                   g1 = vbkey(Hk, (ck) & 0xFFu, 4 * (k) + 1, cont);                                 \
    const bool o4 = (4 * (k) + 4 <= len) & bloom_ok(g4), o3 = (4 * (k) + 3 <= len) & bloom_ok(g3),  \
               o2 = (4 * (k) + 2 <= len) & bloom_ok(g2), o1 = bloom_ok(g1);                         \
    if (o4 | o3 | o2 | o1) fl = o4 ? 4 * (k) + 4 : o3 ? 4 * (k) + 3 : o2 ? 4 * (k) + 2 : 4 * (k) + 1; \
  }
              TOK4_GROUP(5, H5, H6, c5)
              TOK4_GROUP(4, H4, H5, c4)
              TOK4_GROUP(3, H3, H4, c3)
              TOK4_GROUP(2, H2, H3, c2)
              TOK4_GROUP(1, H1, H2, c1)
              TOK4_GROUP(0, H0, H1, c0)
#undef TOK4_GROUP
              if (dbg) acc[7] += len - fl;
              found = fl > 0;
              e = s + fl;
              if (found) hcur = hash_len(fl);  // bucket hash of the survivor only
            } else {
              while (e > s) {
                if (bloom_ok(bkey_len(e - s))) {
                  hcur = hash_len(e - s);
                  found = true;
                  break;
                }
                if (dbg) acc[7] += 1;
                shrink();
              }
            }
            if (found) slot = (int)(hcur & vmask);
            else fail = true;
          }
          STAMP(12);
          if (fail) {  // some position has no match: the whole word is [UNK]
            np = 0;
            put_piece(P.unk);
            finish();
          } else {
            if (dbg) acc[6] += 1;
            const int len = e - s;
            const int lc = min(len, 24), q = lc >> 2, r = lc & 3;
            auto msk = [&](int k, uint32_t c) {  // the key's bytes of dword k, branch-free
              const int nbk = min(max(lc - 4 * k, 0), 4);
              return c & (nbk >= 4 ? 0xFFFFFFFFu : ((1u << (8 * nbk)) - 1u));
            };
            (void)q;
            (void)r;
            const uint32_t m0c = msk(0, c0), m1c = msk(1, c1), m2c = msk(2, c2), m3c = msk(3, c3), m4c = msk(4, c4),
                           m5c = msk(5, c5);
            const uint4* bk = P.vt + 4 * (uint32_t)slot;
            const uint32_t want = ((uint32_t)len << 16) | (cont << 24) | 0x80000000u;
            uint4 a0, a1, b0, b1;
            if (P.dbg_mode == 3) {  // ablation: the survivor "hits" without its bucket load
              a0 = make_uint4(m0c, m1c, m2c, m3c);
              a1 = make_uint4(m4c, m5c, want | 100u, 0u);
              b0 = b1 = make_uint4(0, 0, 0, 0);
            } else {
              a0 = bk[0]; a1 = bk[1]; b0 = bk[2]; b1 = bk[3];
            }
            bool m0 = (((a1.z & 0xFFFF0000u) ^ want) | (a0.x ^ m0c) | (a0.y ^ m1c) | (a0.z ^ m2c) | (a0.w ^ m3c) |
                       (a1.x ^ m4c) | (a1.y ^ m5c)) == 0u;
            bool m1 = (((b1.z & 0xFFFF0000u) ^ want) | (b0.x ^ m0c) | (b0.y ^ m1c) | (b0.z ^ m2c) | (b0.w ^ m3c) |
                       (b1.x ^ m4c) | (b1.y ^ m5c)) == 0u;
            if (m0 && len > 24) m0 = long_eq(L, P, s, len, a1.w);
            if (m1 && len > 24) m1 = long_eq(L, P, s, len, b1.w);
            if (m0 || m1) {
              put_piece((m0 ? a1.z : b1.z) & 0xFFFFu);
              s = e;
              if (s >= we) {
                finish();
              } else {
                cont = 1;
                start_piece(mb1);
              }
            } else if (!(a1.z & 0x80000000u) || !(b1.z & 0x80000000u)) {
              slot = -1;  // an empty slot ends the probe sequence: no such key
              shrink();
            } else {
              slot = (int)(((uint32_t)slot + 1u) & vmask);
            }
          }
        }
        STAMP(13);
        const uint64_t idle = __ballot(u < 0);
        if (next < nwl) {
          if (u < 0) {
            const int r = next + lane_rank(idle);
            if (r < nwl) begin(L.uwp[r]);
          }
          next += __popcll(idle);
        }
        STAMP(14);
      }
    }
    wsync();
    STAMP(4);
    // ---- 5: token positions (segmented scan by sentence) and output ---------
    {
      constexpr int K = UCAP / 64;
      const int per = (nr + 63) >> 6;
      const int u0 = lane * per;
      const int first_sent = (int)(L.urec[0] >> 16);
      const int carry0 = first_sent == prev_sent ? (int)L.stot[first_sent] : 0;
      auto is_head = [&](int uu, int sj) {
        return uu == 0 ? sj != prev_sent : (int)(L.urec[uu - 1] >> 16) != sj;
      };
      int run = 0, head = 0;
      int lpre[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        lpre[k] = 0;
        const int uu = u0 + k;
        if (k < per && uu < nr) {
          const int sj = (int)(L.urec[uu] >> 16);
          if (is_head(uu, sj)) {
            run = 0;
            head = 1;
          }
          lpre[k] = run;
          run += L.ucnt[uu];
        }
      }
      uint32_t hv = (uint32_t)head, sv = (uint32_t)run;
      wave_seg_incl_add(hv, sv);
      int ex = (int)wave_shr1(sv), exh = (int)wave_shr1(hv);  // lane 0: 0
      if (!exh) ex += carry0;  // units before any head continue the previous round's sentence
      bool before = true;
      const int64_t obase = (A - base) - aoff;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int uu = u0 + k;
        if (k < per && uu < nr) {
          const uint32_t rec = L.urec[uu];
          const int sj = (int)(rec >> 16);
          if (is_head(uu, sj)) before = false;
          const int pos = lpre[k] + (before ? ex : 0);
          const int c = L.ucnt[uu];
          uint16_t* out = P.out_ids + (obase + (int64_t)L.sst[sj] + pos);
          const int po = L.pcs.upo[uu];
          // plain stores: L2 merges the partial lines (non-temporal u16
          // stores measured 1 % faster but 7.6x the HBM write bytes)
          if (po == 0xFFFF) {
            if (c > 0 && pos < P.max_tok) out[0] = L.pcs.uid[uu];
          } else {
            for (int q = 0; q < c && pos + q < P.max_tok; ++q) out[q] = L.pcs.mp[po + q];
          }
          if (uu == nr - 1 || (int)(L.urec[uu + 1] >> 16) != sj) L.stot[sj] = (uint16_t)(pos + c);
        }
      }
      wsync();
      prev_sent = (int)(L.urec[nr - 1] >> 16);
      wsync();
    }
    }  // rounds
    if (L.misc[2]) {
      fallback();
      if (dbg) { acc[11] += 1; acc[15] += 1; }
      continue;
    }
    for (int j = lane; j < ns; j += 64) P.out_ntok[sa + j] = min((int)L.stot[j], P.max_tok);
    STAMP(5);
  }
  if (dbg && lane == 0)
    for (int k = 0; k < 16; ++k) atomicAdd((unsigned long long*)&P.dbg[k], (unsigned long long)acc[k]);
#undef STAMP
}

template <int WAVES, bool BLOOM, bool DBG, int H = 1>
hipError_t launch_cfg(const TokParams& P, int64_t n_tiles, const int64_t* tile_sent, int32_t* fb_list,
                      int32_t* fb_count, int n_cu, hipStream_t s) {
  static int per_cu = 0;
  if (per_cu == 0) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, tok4_kernel<WAVES, BLOOM, DBG, H>, 64 * WAVES, 0) !=
            hipSuccess ||
        per_cu < 1)
      per_cu = 1;
  }
  int64_t grid = (int64_t)n_cu * per_cu;
  const int64_t need = ((n_tiles + H - 1) / H + WAVES - 1) / WAVES;
  if (grid > need) grid = need;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL((tok4_kernel<WAVES, BLOOM, DBG, H>), dim3((unsigned)grid), dim3(64 * WAVES), 0, s, P,
                     tile_sent, n_tiles, fb_list, fb_count);
  return hipGetLastError();
}

}  // namespace tok4

hipError_t launch_tokenize_stream(const TokParams& P, int64_t nbytes, int64_t* tile_sent, int32_t* fb_list,
                                  int32_t* fb_count, int fb_grid, int n_cu, int cfg, hipStream_t s) {
  const int64_t n_tiles = tile_count(nbytes);
  hipError_t e = launch_tile_bounds(P.sent_off, P.n_sent, n_tiles, tile_sent, s);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(fb_count, 0, 4, s);
  if (e != hipSuccess) return e;
  if (P.dbg) {  // phase stamps + counters (LDDL_TOK_DEBUG=1), separate instantiation
    e = cfg == 1 ? tok4::launch_cfg<4, false, true>(P, n_tiles, tile_sent, fb_list, fb_count, n_cu, s)
                 : tok4::launch_cfg<4, true, true>(P, n_tiles, tile_sent, fb_list, fb_count, n_cu, s);
  } else {
    switch (cfg) {
      case 1: e = tok4::launch_cfg<4, false, false>(P, n_tiles, tile_sent, fb_list, fb_count, n_cu, s); break;
      case 2: e = tok4::launch_cfg<12, true, false>(P, n_tiles, tile_sent, fb_list, fb_count, n_cu, s); break;
      case 3: e = tok4::launch_cfg<8, true, false>(P, n_tiles, tile_sent, fb_list, fb_count, n_cu, s); break;
      case 4: e = tok4::launch_cfg<16, true, false>(P, n_tiles, tile_sent, fb_list, fb_count, n_cu, s); break;
      case 5: e = tok4::launch_cfg<8, true, false, 2>(P, n_tiles, tile_sent, fb_list, fb_count, n_cu, s); break;
      case 6: e = tok4::launch_cfg<4, true, false, 2>(P, n_tiles, tile_sent, fb_list, fb_count, n_cu, s); break;
      default: e = tok4::launch_cfg<4, true, false>(P, n_tiles, tile_sent, fb_list, fb_count, n_cu, s); break;
    }
  }
  if (e != hipSuccess) return e;
  return launch_tokenize_fallback(P, tile_sent, fb_list, fb_count, fb_grid, s);
}

}  // namespace lddl
