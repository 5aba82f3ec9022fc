// Tokenizer v5 (default): the per-tile scan and WordPiece are split into
// separate kernels so that WordPiece runs at full lane occupancy.
//
// Contract: lddl_tokenize (include/lddl_amd.h); results those of HF
// tokenizers' BertNormalizer / BertPreTokenizer / WordPiece behind
// tokenizer.tokenize(s, max_length=512, truncation=True),
// lddl/dask/bert/pretrain.py:79-80; restated in oracle/tokenizer_oracle.c).
//
// Why: in round 1's one-kernel tile tokenizer (tok4, retired) the WordPiece loop took ~60 %
// of the wave time at ~17 % lane occupancy -- a 1 KiB tile has ~20 words
// that are not whole-word vocab hits, each needing a serial chain of Bloom
// scans and dependent bucket loads, so the wave idled behind the longest
// chain with most lanes masked off.
//
//  scan_kernel     wave per 1 KiB tile (sentences starting in it), persistent:
//                  bytes -> normalised bytes + break masks (per-byte classes, exceptions),
//                  units, dirty words normalised, specials, > 100-char words,
//                  one whole-word bucket probe per unit.  Every unit that
//                  yields tokens becomes an ENTRY of its sentence: a vocab id,
//                  or (a word the probe did not resolve) a reference to a
//                  64-B RECORD {len, count, key bytes} in a chunked queue.
//                  Per sentence: #entries (capped at max_tok: each entry is
//                  >= 1 token), #record slots, first slot, resolved count.
//  wp_kernel       the records, one per lane with refill: greedy
//                  longest-match-first (Bloom scan + 64-B bucket probe per
//                  candidate), pieces and count written back
//                  into the record.
//  expand_kernel   per group of sentences: the entries from each sentence's
//                  first queued word on -> ids (a record's pieces in place of
//                  its entry) and the token count; the ids before it were
//                  final and written by the scan.
// Tiles the scan does not model (window > 2 KiB, > 64 sentences, > 256
// units, a queued word longer than 56 bytes, record capacity) are
// listed and re-run by tokenize_fallback_kernel (exact serial path).
#include <string.h>

#include "common.h"
#include "tokenize.h"
#include "wave.h"
#include "tokenize_serial.h"
#include "pack.h"


namespace lddl {
namespace tok5 {

// (a 1.5 KiB window for 6 waves/SIMD measured slower: 0.2 % of the tiles fall
// back to the serial path, finish 0.97 -> 3.2 ms per GiB, and the 80-VGPR
// scan spills: 3.80 vs 3.49)
// LDDL_PROBE_REC (measurement builds only, results not exact): 1 stores
// only a record's first 16 B, 2 no record bytes (the scan-side bound of
// smaller WordPiece records)
#ifndef LDDL_PROBE_REC
#define LDDL_PROBE_REC 0
#endif
// LDDL_PROBE_L2 (measurement builds only, results not exact): the whole-word
// probe reads 1 MB of the table (L2-resident); 2: and takes every probed word
// as found (no records from probe misses); 3: the whole table, every probed
// word taken as found
#ifndef LDDL_PROBE_L2
#define LDDL_PROBE_L2 0
#endif
constexpr int CAP = 2048;                // window bytes (32 per lane)
constexpr int DCAP = 256;                // side buffer for dirty words
constexpr int SCAN_OCC = 5;              // waves per SIMD the scan's LDS admits (4 measured 5 % slower)
#ifndef LDDL_SCAN_SUPER
#define LDDL_SCAN_SUPER 16
#endif
constexpr int SUPER = LDDL_SCAN_SUPER;   // tiles per super-tile (a wave's unit of hand-out, packed into windows)
#ifndef LDDL_SCAN_FK
#define LDDL_SCAN_FK 2
#endif
constexpr int FK = LDDL_SCAN_FK;         // fast steps per batch (their probe loads in flight together)
#ifndef LDDL_SCAN_FKEY
#define LDDL_SCAN_FKEY 16
#endif
constexpr int FKEY = LDDL_SCAN_FKEY;     // longest key the fast step probes (16 or 24 bytes)
constexpr int NBUF = CAP + DCAP + 64;    // + over-read pad of the key loads
constexpr int UCAP = 256;                // units per round
constexpr int NSCAP = 32;                // sentences per window (< NSCAP: NSCAP sentence offsets staged)
constexpr int XCAP = 32;                 // expansion markers per tile
constexpr int KEYMAX = 56;               // key bytes a record holds
constexpr int KEY1 = 28;                 // keys up to 28 bytes take one slot (<= 28 pieces)
constexpr uint32_t BF = 0xFFu, BX = 0xFDu, BS = 0xF8u;  // filler, expansion, special k = BS+k
// fast exception entry (TokParams::xmap, one per code point; built by
// lddl_create from the unicode table): replacement bytes 0-23, their count
// 24-26, action 27-28, 29 write the replacement, 31 SLOW (the full path)
constexpr uint32_t XM_SLOW = 0x80000000u, XM_WRITE = 0x20000000u;
enum : uint32_t { XM_WORD = 0, XM_SPACE = 1, XM_ISOLATE = 2, XM_DROP = 3 };
__device__ __forceinline__ uint32_t xm_len(uint32_t e) { return (e >> 24) & 7u; }
__device__ __forceinline__ uint32_t xm_act(uint32_t e) { return (e >> 27) & 3u; }
enum : uint32_t { C_W = 1, C_I = 2, C_S = 4, C_D = 8, C_UP = 16, C_X = 32, C_CS = 64 };
constexpr uint16_t U_EMPTY = 0xFFFEu, U_DEFER = 0xFFFFu;


// per lane of the window (LDS, for the unit steps): the first break / dirty
// byte in a later lane and the sentence starts before the lane
__device__ __forceinline__ uint32_t lx_make(int nxt_brk, int nxt_dirty, int sbb) {
  return (uint32_t)nxt_brk | ((uint32_t)nxt_dirty << 12) | ((uint32_t)sbb << 24);
}

struct alignas(16) Lds {
  uint32_t rp[CAP / 4 + 4];    // raw bytes of the tile (LDS-DMA); free after the exception pass, when the
                               // next tile's bytes are prefetched into it
  uint32_t pb[4];              // the next super-tile's bounds: tile_sent of its first tile and of its end (LDS-DMA)
  int64_t soff[NSCAP];         // the next window's sent_off[c_s .. c_s + 32) (LDS-DMA; read by stage2, then its
                               // sentence starts by the window's first steps)
  int64_t wst[4];              // window staging: the super-tile's next sentence, its end, the super-tile, the
                               // next super-tile (kept here, not in registers, across the window's work)
  uint32_t nb[NBUF / 4];       // normalised bytes in window coordinates; side buffer at [CAP, CAP+DCAP)
  uint32_t brk[64];            // break bits: unit starts, spaces, sentence starts
  uint32_t um[64];             // unit-start bits
  uint32_t xm[5 * 64];         // exception pass: every lane's CS, D masks (W, I, S in brk, um, dm), its
                               // SLOW bits, and 256 listed positions (u16); then the unit start
                               // positions of a round (u16, UCAP), lx_make per lane at [128, 192) and
                               // the lanes' unit bases at [256, 320)
  uint32_t dm[64];             // dirty bits: filler / expansion marker bytes
  uint32_t sb[64];             // sentence-start bits
  uint32_t sacc[NSCAP];        // per sentence: its record slots | (queued + empty units) << 16 (LDS atomics
                               // of the rare lanes; direct ids = units - the high half)
  uint16_t sst[NSCAP + 2];     // sentence starts (window coordinates)
  uint16_t ufirst[NSCAP + 2];  // index of the sentence's first unit in the tile ([ns] = #units)
  uint16_t ebs[NSCAP];         // entry index base: unit u of sentence j has entry sst[j] + u - ufirst[j]
  uint32_t xrep[XCAP * 3];     // each expansion marker's normalised bytes (<= 12: up to three chars)
  uint8_t xlen[XCAP];          // their number
  int32_t misc[4];             // 0 side-buffer cursor, 1 #markers
  uint32_t sspec[2];           // sentences holding a [CLS] / [SEP] token (P.sent_spec)
};

// SCAN_OCC 4-wave blocks per CU (+ the 256-B class table): SCAN_OCC waves per SIMD
static_assert(4 * sizeof(Lds) + 256 <= 160 * 1024 / SCAN_OCC, "scan LDS no longer admits SCAN_OCC waves per SIMD");

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// LDS-DMA (global_load_lds: lane i's bytes land at the LDS base + i * size,
// M0 = the LDS base) issued from inline asm.  The compiler's wait insertion
// does not see these loads, so it places no conservative vmcnt wait before
// every later LDS read (it cannot tell the DMA's target from the arrays the
// window's steps read, and a wait there also waits for every probe load in
// flight); the scan drains them itself (drain(): s_waitcnt vmcnt(0)) before
// it reads what they wrote.  vmcnt counts in issue order, so a wait the
// compiler places for one of its own loads stays correct: an unseen younger
// DMA only makes it stricter.  M0 is saved and restored around the load.
__device__ __forceinline__ void lds_dma4(const void* g, uint32_t* l) {
  uint32_t t;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(t)
               : "v"(g), "s"((uint32_t)(uintptr_t)l)
               : "memory");
}
__device__ __forceinline__ void lds_dma16_nt(const void* g, uint32_t* l) {
  uint32_t t;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(t)
               : "v"(g), "s"((uint32_t)(uintptr_t)l)
               : "memory");
}
// record slot k (of 4 16-B quarters) of slot i, quarter-major: the lanes of a
// refill, on consecutive slots, load one contiguous run per quarter
__device__ __forceinline__ uint4* recq(const SplitParams& S, int k, uint64_t i) {
  return S.rec + (uint64_t)k * ((uint64_t)S.n_chunks * SPLIT_CHUNK) + i;
}
__device__ __forceinline__ uint32_t rawb(const Lds& L, int p) { return reinterpret_cast<const uint8_t*>(L.rp)[p]; }
__device__ __forceinline__ uint32_t nbyte(const uint32_t* nb, int p) { return reinterpret_cast<const uint8_t*>(nb)[p]; }
__device__ __forceinline__ void nput(uint32_t* nb, int p, uint32_t v) { reinterpret_cast<uint8_t*>(nb)[p] = (uint8_t)v; }

// bit q of each byte of c -> 4 bits (byte 0 -> bit 0)
__device__ __forceinline__ uint32_t gather4(uint32_t c, int q) { return (((c >> q) & 0x01010101u) * 0x01020408u) >> 24; }

// byte j of a_k -> byte k of t_j (a 4x4 byte transpose, v_perm_b32)
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}
__device__ __forceinline__ void byte_transpose4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t& t0,
                                                uint32_t& t1, uint32_t& t2, uint32_t& t3) {
  const uint32_t l01 = perm(a1, a0, 0x05010400u), h01 = perm(a1, a0, 0x07030602u);  // a0.b0 a1.b0 a0.b1 a1.b1 | .b2 .b3
  const uint32_t l23 = perm(a3, a2, 0x05010400u), h23 = perm(a3, a2, 0x07030602u);
  t0 = perm(l23, l01, 0x05040100u);
  t1 = perm(l23, l01, 0x07060302u);
  t2 = perm(h23, h01, 0x05040100u);
  t3 = perm(h23, h01, 0x07060302u);
}
// bit q of byte k of t_j -> bit 4k + j (16 positions)
__device__ __forceinline__ uint32_t class_plane16(uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3, int q) {
  uint32_t m = (t0 >> q) & 0x01010101u;
  m |= ((t1 >> q) & 0x01010101u) << 1;
  m |= ((t2 >> q) & 0x01010101u) << 2;
  m |= ((t3 >> q) & 0x01010101u) << 3;  // bit 8k + j
  m = (m | (m >> 4)) & 0x00FF00FFu;
  return (m | (m >> 8)) & 0xFFFFu;
}

// the lane index, re-materialised where it is used: per-lane 64-bit address
// offsets (lane * 8 ...) derived from it are otherwise hoisted out of the
// tile loop and spilled, and a spill reload's vmcnt(0) then waits for the
// next tile's prefetched bytes as well
__device__ __forceinline__ int lane_here() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
__device__ __forceinline__ int64_t uni64(int64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int lane_rank(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ int utf8_put(uint32_t* nb, int p, uint32_t c) {
  if (c < 0x80) { nput(nb, p, c); return 1; }
  if (c < 0x800) { nput(nb, p, 0xC0 | (c >> 6)); nput(nb, p + 1, 0x80 | (c & 0x3F)); return 2; }
  if (c < 0x10000) {
    nput(nb, p, 0xE0 | (c >> 12)); nput(nb, p + 1, 0x80 | ((c >> 6) & 0x3F)); nput(nb, p + 2, 0x80 | (c & 0x3F));
    return 3;
  }
  nput(nb, p, 0xF0 | (c >> 18)); nput(nb, p + 1, 0x80 | ((c >> 12) & 0x3F));
  nput(nb, p + 2, 0x80 | ((c >> 6) & 0x3F)); nput(nb, p + 3, 0x80 | (c & 0x3F));
  return 4;
}

// Compact / expand the dirty span [p, q).  Returns its normalised length
// (source in *src), -1 on overflow (the tile falls back).  Without expansion
// markers in the tile (misc[1] == 0) a dirty span holds only fillers
// (dropped / shortened chars): it compacts in place, one pass; otherwise it
// goes to the side buffer (count pass, then the expansions written).
__device__ int dirty_normalize(Lds& L, const TokParams& P, int p, int q, int* src) {
  if (L.misc[1] == 0) {
    // dword reads (no read waits on the previous byte's write: a byte is
    // written at or below the position read, never into a later dword)
    int o = p;
    for (int a = p & ~3; a < q; a += 4) {
      const uint32_t v = L.nb[a >> 2];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t b = (v >> (8 * k)) & 0xFFu;
        if (a + k >= p && a + k < q && b != BF) nput(L.nb, o++, b);
      }
    }
    *src = p;
    return o - p;
  }
  // (dword reads here too: one LDS round trip per 4 bytes instead of one per
  // byte; a marker's index byte may sit in the next dword: `skip` carries it)
  int len = 0;
  bool skip = false;
  for (int a = p & ~3; a < q; a += 4) {
    const uint32_t v = L.nb[a >> 2];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t b = (v >> (8 * k)) & 0xFFu;
      if (a + k < p || a + k >= q) continue;
      if (skip) {
        len += L.xlen[b];
        skip = false;
      } else if (b == BX) {
        skip = true;
      } else if (b != BF) {
        ++len;
      }
    }
  }
  if (len == 0) return 0;
  const int off = atomicAdd(&L.misc[0], len);
  if (off + len > DCAP) return -1;
  int o = CAP + off;
  *src = o;
  // (the side buffer lies past CAP, beyond every span read here)
  skip = false;
  for (int a = p & ~3; a < q; a += 4) {
    const uint32_t v = L.nb[a >> 2];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t b = (v >> (8 * k)) & 0xFFu;
      if (a + k < p || a + k >= q) continue;
      if (skip) {
        // (the marker's bytes, encoded when the exception pass placed it: no
        // table load here)
        const int nx = L.xlen[b];
        for (int t = 0; t < nx; ++t) nput(L.nb, o++, nbyte(L.xrep, 12 * (int)b + t));
        skip = false;
      } else if (b == BX) {
        skip = true;
      } else if (b != BF) {
        nput(L.nb, o++, b);
      }
    }
  }
  return len;
}

__device__ __forceinline__ int count_chars(const uint32_t* nb, int src, int len) {
  int n = 0;
  for (int i = 0; i < len; ++i) n += (nbyte(nb, src + i) & 0xC0u) != 0x80u;
  return n;
}

// the first min(len, 24) bytes at s as six little-endian dwords, zero beyond
struct Key6 {
  uint32_t d0, d1, d2, d3, d4, d5;
};
__device__ __forceinline__ uint32_t keep_bytes(uint32_t c, int rem) {
  return rem >= 4 ? c : rem <= 0 ? 0u : (c & ((1u << (8 * rem)) - 1u));
}
__device__ __forceinline__ Key6 load_key(const uint32_t* nb, int s, int len) {
  const int a = s >> 2;
  const uint32_t sh = (uint32_t)(s & 3);
  const uint32_t x0 = nb[a], x1 = nb[a + 1], x2 = nb[a + 2], x3 = nb[a + 3], x4 = nb[a + 4], x5 = nb[a + 5],
                 x6 = nb[a + 6];
  const int lc = min(len, 24);
  Key6 k;
  k.d0 = keep_bytes(__builtin_amdgcn_alignbyte(x1, x0, sh), lc);
  k.d1 = keep_bytes(__builtin_amdgcn_alignbyte(x2, x1, sh), lc - 4);
  k.d2 = keep_bytes(__builtin_amdgcn_alignbyte(x3, x2, sh), lc - 8);
  k.d3 = keep_bytes(__builtin_amdgcn_alignbyte(x4, x3, sh), lc - 12);
  k.d4 = keep_bytes(__builtin_amdgcn_alignbyte(x5, x4, sh), lc - 16);
  k.d5 = keep_bytes(__builtin_amdgcn_alignbyte(x6, x5, sh), lc - 20);
  return k;
}
// the first min(len, 16) bytes at s, zero beyond (d4 = d5 = 0): the fast
// step's key (a whole word of <= 16 bytes: five LDS reads, four byte aligns)
__device__ __forceinline__ Key6 load_key16(const uint32_t* nb, int s, int len) {
  const int a = s >> 2;
  const uint32_t sh = (uint32_t)(s & 3);
  const uint32_t x0 = nb[a], x1 = nb[a + 1], x2 = nb[a + 2], x3 = nb[a + 3], x4 = nb[a + 4];
  const int lc = min(len, 16);
  Key6 k;
  k.d0 = keep_bytes(__builtin_amdgcn_alignbyte(x1, x0, sh), lc);
  k.d1 = keep_bytes(__builtin_amdgcn_alignbyte(x2, x1, sh), lc - 4);
  k.d2 = keep_bytes(__builtin_amdgcn_alignbyte(x3, x2, sh), lc - 8);
  k.d3 = keep_bytes(__builtin_amdgcn_alignbyte(x4, x3, sh), lc - 12);
  k.d4 = k.d5 = 0;
  return k;
}
// a value the optimiser cannot see through: keeps the xor / or reduction
// below (v_xor + v_or3) from being rewritten into one compare per dword,
// materialised bools and 16-bit shifts
__device__ __forceinline__ uint32_t opq(uint32_t x) {
  asm("" : "+v"(x));
  return x;
}
// == vhash (common.h) of a loaded key; branch-free: the six mixes, then the
// one of the key's length selected (a branch per dword diverges across lanes)
__device__ __forceinline__ uint32_t key_hash(const Key6& k, int len, uint32_t cont) {
  return vfinal(vmix(vmix(vmix(VSEED, k.d0), k.d1), k.d2), (uint32_t)len, cont);  // (key dwords zero past len)
}
// branch-free (an && chain lets the compiler sink the slot's other loads
// behind the first compare: a second dependent round trip on every hit)
__device__ __forceinline__ bool slot_eq(const uint4& a, const uint4& b, const Key6& k, uint32_t want) {
  const uint32_t d = opq((b.z & 0xFFFF0000u) ^ want) | opq(a.x ^ k.d0) | opq(a.y ^ k.d1) | opq(a.z ^ k.d2) |
                     opq(a.w ^ k.d3) | opq(b.x ^ k.d4) | opq(b.y ^ k.d5);
  return d == 0u;
}

// DBG: phase stamps (s_memtime, diagnostics build only: LDDL_TOK_DEBUG=1)
// OCC: the waves per SIMD the register allocation is held to (LDS admits 5)
template <int WAVES, bool DBG, int OCC>
__global__ __launch_bounds__(64 * WAVES, OCC) void scan_kernel(TokParams P, SplitParams S) {
  uint64_t acc[17] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tprev = 0;
#define STAMP(k)                                                                   \
  if (DBG) {                                                                       \
    uint64_t t_;                                                                   \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");   \
    acc[k] += t_ - tprev;                                                          \
    tprev = t_;                                                                    \
  }
  __shared__ Lds Ls[WAVES];
  __shared__ uint32_t ctab32[64];
  // ---- prologue: per-byte class table from the unicode table's ASCII page --
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
  __syncthreads();
  const uint8_t* ctab = reinterpret_cast<const uint8_t*>(ctab32);
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  Lds& L = Ls[wv];
  const int64_t base = P.sent_off[0];
  const int64_t ebase = S.t0 << 10;  // entry index = byte offset (from base) - ebase
  const int64_t nwaves = (int64_t)gridDim.x * WAVES;
  const int max_tok = P.max_tok;
  // record chunk of this wave (wave-uniform): slots [cur, cend)
  uint32_t cur = 0, cend = 0, cbase = 0, tbase = 0, tsl = 0;
  int chunk = -1;
  // Windows.  The wave walks super-tiles of SUPER tiles (its wave index, then
  // the ones it claims from a counter) and packs each one's sentences greedily into windows: as many
  // whole sentences (<= 63) as fit in CAP bytes from the first one's 16-B
  // aligned start.  A window is about twice a tile's bytes, so the per-window
  // work (classification, exception pass, unit scans, per-sentence records)
  // runs over a nearly full 2 KiB window instead of a ~1 KiB tile in it.  A
  // sentence longer than the window is a window of its own and falls back.
  // The next window is staged inside the current one: stage1 loads
  // sent_off[c_s + lane] (its sentences' starts and ends) right after this
  // window's own bytes arrived, stage2 (before this window's unit steps)
  // finds how many sentences fit and moves their raw bytes into rp (free
  // after this window's exception pass) by LDS-DMA, so both round trips fly
  // behind this window's work; the loop top finishes whatever a window that
  // returned early left undone.  A super-tile's bounds (tile_sent) arrive by
  // LDS-DMA into pb while the one before it runs.  Super-tiles past the
  // first are claimed from a per-segment counter (chunk_ctr[2]) one
  // transition ahead (the claim's return is read at the next transition), so
  // a wave that starts late -- its CU still busy with another kernel's waves
  // -- takes fewer of them instead of finishing the launch late.  A wave
  // claims only what it will run: a claim made after another is larger, so
  // when a wave's next super-tile is past the end, so is every one it holds.
  int64_t n_sa = 0, n_sb = 0, n_A = 0, n_B = 0;
  int nst = 0;
  bool dma_pending = false;  // raw-byte DMA issued and not yet waited for
  const int64_t ng = (S.t1 - S.t0 + SUPER - 1) / SUPER;
  // (LDS-DMA: lane i of the instruction writes dword i at the LDS base)
  auto dma4 = [&](const void* g, uint32_t* l) { lds_dma4(g, l); };
  auto drain = [&]() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };
  // (lanes 0-1: tile_sent of super-tile g's first tile, lanes 2-3: of its end -> pb[0..3])
  auto st_bounds = [&](int64_t g) {
    if (g < ng && lane < 4) {
      const int64_t t = min(S.t1, S.t0 + (g + (lane >> 1)) * SUPER);
      dma4(reinterpret_cast<const uint32_t*>(S.tile_sent + t) + (lane & 1), L.pb);
    }
  };
  uint32_t* const sctr = S.chunk_ctr + 2;  // zeroed with chunk_ctr per segment
  uint32_t gq = 0;                         // lane 0: the claim after the next super-tile (in flight)
  auto claim = [&]() {
    if (lane == 0) gq = atomicAdd(sctr, 1u);
  };
  {
    const int64_t g = (int64_t)blockIdx.x * WAVES + wv;
    int64_t cs = 0, ce = 0, gn = ng;
    if (g < ng) {
      cs = uni64(S.tile_sent[S.t0 + g * SUPER]);
      ce = uni64(S.tile_sent[min(S.t1, S.t0 + (g + 1) * SUPER)]);
      claim();
      gn = nwaves + (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)gq, 0);
      claim();
    }
    L.wst[0] = cs;
    L.wst[1] = ce;
    L.wst[2] = g;
    L.wst[3] = gn;
    wsync();
    st_bounds(gn);
  }
  auto stage1 = [&]() {
    if (nst != 0) return;
    nst = 1;
    int64_t cs = uni64(L.wst[0]), ce = uni64(L.wst[1]), g = uni64(L.wst[2]);
    if (cs >= ce && g < ng) {
      int64_t gn = uni64(L.wst[3]);
      while (cs >= ce && g < ng) {  // the super-tile is done: the next one's bounds (pb)
        g = gn;
        if (g >= ng) break;
        drain();
        cs = uni64(*reinterpret_cast<const int64_t*>(&L.pb[0]));
        ce = uni64(*reinterpret_cast<const int64_t*>(&L.pb[2]));
        gn = nwaves + (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)gq, 0);
        claim();
        st_bounds(gn);
      }
      L.wst[0] = cs;
      L.wst[1] = ce;
      L.wst[2] = g;
      L.wst[3] = gn;
    }
    // (lane l: dword l of sent_off[cs ..], the offsets up to ce)
    if (cs < ce && cs + (lane_here() >> 1) <= ce) dma4(reinterpret_cast<const uint32_t*>(P.sent_off + cs) + lane_here(), reinterpret_cast<uint32_t*>(L.soff));
  };
  auto stage2 = [&]() {
    if (nst != 1) return;
    nst = 2;
    n_sa = n_sb = 0;
    const int64_t cs = uni64(L.wst[0]), ce = uni64(L.wst[1]);
    if (cs >= ce) return;
    drain();
    const int64_t a = uni64(L.soff[0]);
    const int aoff = (int)(reinterpret_cast<uintptr_t>(P.bytes + a) & 15u);
    // (sentence i < NSCAP - 1 of the window ends at offset i + 1: a prefix of the lanes fits)
    const int ln = lane_here();
    const bool in = ln >= 1 && ln < NSCAP && cs + ln <= ce;
    const uint64_t fit = __ballot(in && L.soff[in ? ln : 0] <= a - aoff + CAP);
    const int ns = max((int)__popcll(fit), 1);  // (0: the first sentence alone is longer; it falls back)
    n_sa = cs;
    n_sb = cs + ns;
    n_A = a;
    n_B = uni64(L.soff[ns]);
    L.wst[0] = cs + ns;
    const int64_t nb64 = (n_B - n_A) + aoff;
    if (nb64 > CAP) return;  // the window falls back: no bytes needed
    dma_pending = true;
    // streamed once: non-temporal (aux bit 1), keep L2 for the vocab table
    const uint8_t* g = P.bytes + (n_A - aoff) + 16 * ln;
    if (16 * ln < nb64) lds_dma16_nt(g, L.rp);
    if (1024 + 16 * ln < nb64) lds_dma16_nt(g + 1024, L.rp + 256);
  };
  if (DBG) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tprev)::"memory");
  for (;;) {
    wsync();
    stage1();
    stage2();
    if (n_sa >= n_sb) break;  // no window left
    const int64_t sa = n_sa, sb = n_sb, A = n_A, B = n_B;
    STAMP(0);
    if (dma_pending) drain();  // this window's raw bytes
    dma_pending = false;
    nst = 0;
    [&]() {
    if (sa >= sb) return;
    const int ns = (int)(sb - sa);
    // the window goes to the exact serial kernel; its sentences are no-ops for
    // the count / expand passes
    auto fallback = [&]() {
      if (lane == 0) {
        const int at = atomicAdd(S.fb_count, 1);
        S.fb_list[2 * at] = sa;
        S.fb_list[2 * at + 1] = sb;
        atomicAdd(S.n_fallback, 1u);
      }
      for (int j = lane_here(); j < ns; j += 64) {
        S.smeta[sa + j] = make_uint2(SPLIT_NENT_FB, 0xFFFFFFFFu);
      }
    };
    const int aoff = (int)(reinterpret_cast<uintptr_t>(P.bytes + A) & 15u);
    const uint8_t* wbase = P.bytes + (A - aoff);  // 16-B aligned
    const int64_t nb64 = (B - A) + aoff;
    if (nb64 > CAP || ns > NSCAP) {
      fallback();
      return;
    }
    const int nb = (int)nb64;
    // ---- sentence starts ----------------------------------------------------
    L.sb[lane] = 0;
    if (lane == 0) {
      L.misc[0] = 0;
      L.misc[1] = 0;
      L.sspec[0] = 0;
      L.sspec[1] = 0;
    }
    if (lane < ns) L.sacc[lane] = 0;
    wsync();
    if (lane < ns) {
      const int pos = (int)(L.soff[lane] - A) + aoff;
      L.sst[lane] = (uint16_t)pos;
      if (pos < nb) atomicOr(&L.sb[pos >> 5], 1u << (pos & 31));
    }
    wsync();
    stage1();  // (soff is read: the next window's offsets may land)
    STAMP(1);
    // ---- 1: raw bytes -> masks + normalised bytes in place ------------------
    uint32_t W, I, S_, CS, D, X, inwin;
    {
      const int p0 = lane * 32;
      (void)wbase;  // the raw bytes came with the prefetch (stage3), bytes >= nb zero
      uint4 v0 = make_uint4(0, 0, 0, 0), v1 = v0;
      if (p0 < CAP) {
        v0 = *reinterpret_cast<const uint4*>(&L.rp[lane * 8]);
        v1 = *reinterpret_cast<const uint4*>(&L.rp[lane * 8 + 4]);
      }
      if (p0 >= nb) v0 = make_uint4(0, 0, 0, 0);
      if (p0 + 16 >= nb) v1 = make_uint4(0, 0, 0, 0);
      const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      // class bytes c[k] (byte j = position 4k + j), then the per-position
      // class bits as 32-bit planes without multiplies: 4x4 byte transposes
      // put position 4k + j at byte k of t[j]; a plane gathers bit q of the
      // four t[j] (bit 8k + j) and compresses the nibbles (bit 4k + j)
      uint32_t c[8], nv[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t x = w[k];
        c[k] = (uint32_t)ctab[x & 0xFFu] | ((uint32_t)ctab[(x >> 8) & 0xFFu] << 8) |
               ((uint32_t)ctab[(x >> 16) & 0xFFu] << 16) | ((uint32_t)ctab[x >> 24] << 24);
        const uint32_t dmk = (c[k] >> 3) & 0x01010101u;  // drop bytes -> filler 0xFF
        nv[k] = (x + ((c[k] & 0x10101010u) << 1)) | ((dmk << 8) - dmk);
      }
      // two 16-B stores per lane (8 dword stores at a 32-B lane stride hit
      // 1/8 of the banks)
      if (p0 < CAP) {
        *reinterpret_cast<uint4*>(&L.nb[lane * 8]) = make_uint4(nv[0], nv[1], nv[2], nv[3]);
        *reinterpret_cast<uint4*>(&L.nb[lane * 8 + 4]) = make_uint4(nv[4], nv[5], nv[6], nv[7]);
      }
      uint32_t t[8];
      byte_transpose4(c[0], c[1], c[2], c[3], t[0], t[1], t[2], t[3]);
      byte_transpose4(c[4], c[5], c[6], c[7], t[4], t[5], t[6], t[7]);
      auto plane = [&](int q) {
        return class_plane16(t[0], t[1], t[2], t[3], q) | (class_plane16(t[4], t[5], t[6], t[7], q) << 16);
      };
      const uint32_t Wh = plane(0), Ih = plane(1), Sh = plane(2), Dh = plane(3), Xh = plane(5);
      const uint32_t CSh = Wh | Ih | Sh | Xh;  // every byte but UTF-8 continuations (ctab)
      const int wlo = min(max(aoff - p0, 0), 32), whi = min(max(nb - p0, 0), 32);
      inwin = (whi >= 32 ? ~0u : ((1u << whi) - 1u)) & (wlo >= 32 ? 0u : ~((1u << wlo) - 1u));
      W = Wh; I = Ih; S_ = Sh; CS = CSh; D = Dh; X = Xh & inwin;
    }
    wsync();
    STAMP(2);
    bool bad = false;
    uint32_t sp_m = 0, sp_w = 0, sp_d = 0;  // this lane's last char / special running into the next lane
    {
      const int p0 = lane * 32;
      // Fast path over the tile's exception bytes in ONE pass, one per lane
      // (one table round trip for up to 64): the lanes list their exception
      // positions, then lane k takes the k-th -- '[' (a literal special
      // token?) from the raw bytes and the sentence-start bits, a UTF-8 lead
      // byte from one load of its code point's fast entry (xmap: class,
      // replacement bytes, drop) -- and applies it to the owner lanes' masks
      // held in LDS (atomic or / and: a span may run into the next lane).
      // What it does not model (SLOW: multi-char expansions, canonical
      // reordering, a replacement longer than the source) goes back to the
      // owner lane for the full path below.
      uint32_t xslow = 0;
      if (__any(X != 0)) {
        // masks q = 0..4 (W, I, S, CS, D) of lane l at mw(q)[l]; the listed
        // positions (u16) after the SLOW bits
        auto mw = [&](int q) -> uint32_t* { return q == 0 ? L.brk : q == 1 ? L.um : q == 2 ? L.dm : L.xm + (q - 3) * 64; };
        uint32_t* const slowm = L.xm + 128;
        uint16_t* const xl = reinterpret_cast<uint16_t*>(L.xm + 192);
        constexpr uint32_t XL = 256;
        mw(0)[lane] = W;
        mw(1)[lane] = I;
        mw(2)[lane] = S_;
        mw(3)[lane] = CS;
        mw(4)[lane] = D;
        slowm[lane] = 0;
        const uint32_t cx = (uint32_t)__popc(X);
        const uint32_t xi = wave_incl_add(cx);
        const uint32_t nx = lane_get(xi, 63);
        wsync();
        auto mor = [&](int q, int pos, uint32_t nbits) {  // bits [pos, pos + nbits) of mask q
          const int wq = pos >> 5, bq = pos & 31;
          const uint64_t m = ((1ull << nbits) - 1ull) << bq;
          atomicOr(&mw(q)[wq], (uint32_t)m);
          if ((m >> 32) && wq < 63) atomicOr(&mw(q)[wq + 1], (uint32_t)(m >> 32));
        };
        auto mclr = [&](int q, int pos, uint32_t nbits) {
          const int wq = pos >> 5, bq = pos & 31;
          const uint64_t m = ((1ull << nbits) - 1ull) << bq;
          atomicAnd(&mw(q)[wq], ~(uint32_t)m);
          if ((m >> 32) && wq < 63) atomicAnd(&mw(q)[wq + 1], ~(uint32_t)(m >> 32));
        };
        bool any_slow = false;
        for (uint32_t kb = 0; kb < nx; kb += XL) {
          {  // list the exceptions kb .. kb + XL in lane order
            uint32_t k = xi - cx;
            for (uint32_t m = X; m; m &= m - 1, ++k)
              if (k >= kb && k < kb + XL) xl[k - kb] = (uint16_t)(p0 + __ffs(m) - 1);
          }
          wsync();
          STAMP(14);
          const uint32_t nl = min(nx - kb, XL);
        for (uint32_t k0 = 0; k0 < nl; k0 += 64) {
          const uint32_t k = k0 + lane;
          const int p = k < nl ? (int)xl[k] : 0;
          uint32_t e = XM_SLOW, n = 0;
          bool brk = false;
          if (k < nl) {
            const uint32_t b = rawb(L, p);
            if (b == '[') {
              brk = true;
            } else {
              n = (uint32_t)utf8_len(b);
              uint32_t cp = b & (0x3Fu >> (n - 1));
              for (uint32_t q = 1; q < n; ++q) cp = (cp << 6) | (rawb(L, p + (int)q) & 0x3Fu);
              if (cp > 0x10FFFF) cp = 0xFFFD;
              e = P.xmap[cp];
            }
          }
          if (DBG) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          STAMP(15);
          if (brk) {  // [PAD] [UNK] [CLS] [SEP] [MASK] within p's sentence
            const int a = (p + 1) >> 2;
            const uint32_t sh = (uint32_t)((p + 1) & 3);
            const uint32_t w0 = __builtin_amdgcn_alignbyte(L.rp[a + 1], L.rp[a], sh);  // bytes p+1 .. p+4
            const uint32_t w1 = __builtin_amdgcn_alignbyte(L.rp[a + 2], L.rp[a + 1], sh) & 0xFFu;  // byte p+5
            // sentence starts at p+1 .. p+5 end p's sentence (no special crosses one)
            const int wq = (p + 1) >> 5;
            const uint64_t sbw = (uint64_t)L.sb[wq] | ((uint64_t)(wq + 1 < 64 ? L.sb[wq + 1] : 0u) << 32);
            const uint32_t nxt = (uint32_t)(sbw >> ((p + 1) & 31)) & 0x1Fu;
            int len = 0, sk = -1;
            if (p + 5 <= nb && (nxt & 0xFu) == 0) {
              if (w0 == 0x5D444150u) { sk = 0; len = 5; }         // PAD]
              else if (w0 == 0x5D4B4E55u) { sk = 1; len = 5; }    // UNK]
              else if (w0 == 0x5D534C43u) { sk = 2; len = 5; }    // CLS]
              else if (w0 == 0x5D504553u) { sk = 3; len = 5; }    // SEP]
              else if (w0 == 0x4B53414Du && w1 == ']' && p + 6 <= nb && (nxt & 0x10u) == 0) { sk = 4; len = 6; }  // MASK]
            }
            if (sk >= 0) {
              nput(L.nb, p, BS + (uint32_t)sk);
              for (int q = 0; q < 5; ++q) mclr(q, p + 1, (uint32_t)len - 1u);
            }
          } else if (k < nl) {
            if ((e & XM_SLOW) || xm_len(e) > n) {
              any_slow = true;  // (back to the owner lane: xslow)
              atomicOr(&slowm[p >> 5], 1u << (p & 31));
            } else {
              const uint32_t act = xm_act(e), T = xm_len(e);
              bool dirty = false, wordc = false;
              if (act == XM_DROP) {
                for (uint32_t q = 0; q < n; ++q) nput(L.nb, p + (int)q, BF);
                dirty = wordc = true;
              } else if (act == XM_SPACE) {
                mor(2, p, 1);
              } else {
                if (act == XM_ISOLATE) mor(1, p, 1);
                else wordc = true;
                if (e & XM_WRITE) {
                  for (uint32_t q = 0; q < n; ++q) nput(L.nb, p + (int)q, q < T ? (e >> (8 * q)) & 0xFFu : BF);
                  dirty = T < n;
                }
              }
              // (the continuation bytes past this lane carry no class bits)
              if (wordc) mor(0, p, n);
              if (dirty) mor(4, p, n);
            }
          }
        }
          wsync();
        }
        W = mw(0)[lane];
        I = mw(1)[lane];
        S_ = mw(2)[lane];
        CS = mw(3)[lane];
        D = mw(4)[lane];
        if (__any(any_slow)) xslow = slowm[lane];
        STAMP(16);
      }
      // the full path: exceptions in batches of 4 per lane, the table lookups
      // of a batch (code point -> page -> entry -> multi expansion) together
      for (uint32_t xm = xslow; __any(xm != 0);) {
        constexpr int XB = 4;
        int xi_[XB];
        uint32_t xcp[XB], xt[XB], xe[XB];
        uint4 xmul[XB];
#pragma unroll
        for (int j = 0; j < XB; ++j) {
          xi_[j] = -1;
          xcp[j] = 0;
          if (xm) {
            const int i = __ffs(xm) - 1;
            xm &= xm - 1;
            xi_[j] = i;
            const int p = p0 + i;
            const uint32_t b = rawb(L, p);
            if (b != '[') {
              const int n = utf8_len(b);
              uint32_t cp = b & (0x3Fu >> (n - 1));
              for (int q = 1; q < n; ++q) cp = (cp << 6) | (rawb(L, p + q) & 0x3Fu);
              if (cp > 0x10FFFF) cp = 0xFFFD;
              xcp[j] = cp | 0x80000000u;  // (flag: a char, not '[')
            }
          }
        }
        // (code points of the BMP: one load from the flat table; above it, top -> page)
#pragma unroll
        for (int j = 0; j < XB; ++j) xt[j] = (xcp[j] >> 31) && (xcp[j] & 0x1FFFFFu) >= 0x10000u ? (uint32_t)P.top[(xcp[j] & 0x1FFFFFu) >> 8] : 0u;
#pragma unroll
        for (int j = 0; j < XB; ++j) {
          const uint32_t cp = xcp[j] & 0x1FFFFFu;
          xe[j] = !(xcp[j] >> 31) ? 0u : cp < 0x10000u ? P.bmp[cp] : P.pages[xt[j] * 256u + (cp & 255u)];
        }
#pragma unroll
        for (int j = 0; j < XB; ++j)
          xmul[j] = (xcp[j] >> 31) && ent_kind(xe[j]) == KIND_MULTI ? P.multi[ent_payload(xe[j])] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < XB; ++j) {
          if (xi_[j] < 0) continue;
          const int i = xi_[j];
          const int p = p0 + i;
          const uint32_t b = rawb(L, p);
          if (!(xcp[j] >> 31)) {  // '['
            int se = nb;  // end of p's sentence
            for (int jj = 1; jj < ns; ++jj)
              if (L.sst[jj] > p) { se = L.sst[jj]; break; }
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
              nput(L.nb, p, BS + (uint32_t)sk);
              const uint64_t cov = ((1ull << (len - 1)) - 1ull) << (i + 1);
              const uint32_t cl = (uint32_t)cov;
              W &= ~cl;
              I &= ~cl;
              S_ &= ~cl;
              CS &= ~cl;
              D &= ~cl;
              sp_m |= (uint32_t)(cov >> 32);
            }
            continue;
          }
          const int n = utf8_len(b);
          const uint32_t e = xe[j];
          const uint32_t kind = ent_kind(e), cls = ent_cls(e);
          const uint64_t span = ((1ull << n) - 1ull) << i;
          bool dirty = false, wordc = false;
          if (ent_rank(e) != 0) bad = true;
          if (kind == KIND_DROP_T || kind == KIND_DROP_D) {
            for (int q = 0; q < n; ++q) nput(L.nb, p + q, BF);
            dirty = true;
            wordc = true;
          } else if (cls == CLS_SPACE) {
            S_ |= 1u << i;
          } else {
            if (cls == CLS_ISOLATE) I |= 1u << i;
            else wordc = true;
            if (kind != KIND_IDENT) {
              uint32_t c0 = ent_payload(e), c1 = 0, c2 = 0;
              int nc = 1;
              if (kind == KIND_MULTI) {
                const uint4 m = xmul[j];
                nc = (int)m.x;
                c0 = ent_payload(m.y);
                c1 = ent_payload(m.z);
                c2 = ent_payload(m.w);
                if ((ent_rank(m.y) | ent_rank(m.z) | (nc > 2 ? ent_rank(m.w) : 0u)) != 0) bad = true;
              }
              const int T = utf8_enc_len(c0) + (nc > 1 ? utf8_enc_len(c1) : 0) + (nc > 2 ? utf8_enc_len(c2) : 0);
              if (T <= n) {
                int o = p + utf8_put(L.nb, p, c0);
                if (nc > 1) o += utf8_put(L.nb, o, c1);
                if (nc > 2) o += utf8_put(L.nb, o, c2);
                for (; o < p + n; ++o) nput(L.nb, o, BF);
                dirty = T < n;
              } else {
                const int xi = atomicAdd(&L.misc[1], 1);
                if (xi >= XCAP) {
                  bad = true;
                } else {
                  int ox = 12 * xi;
                  ox += utf8_put(L.xrep, ox, c0);
                  if (nc > 1) ox += utf8_put(L.xrep, ox, c1);
                  if (nc > 2) ox += utf8_put(L.xrep, ox, c2);
                  L.xlen[xi] = (uint8_t)T;
                  nput(L.nb, p, BX);
                  nput(L.nb, p + 1, (uint32_t)xi);
                  for (int q = 2; q < n; ++q) nput(L.nb, p + q, BF);
                }
                dirty = true;
              }
            }
          }
          const uint32_t slo = (uint32_t)span, shi = (uint32_t)(span >> 32);
          if (wordc) {
            W |= slo;
            sp_w |= shi;
          }
          if (dirty) {
            D |= slo;
            sp_d |= shi;
          }
          sp_m |= shi;
        }
      }
    }
    {
      const uint32_t im = wave_shr1(sp_m), iw = wave_shr1(sp_w), id = wave_shr1(sp_d);  // lane 0: 0
      W = ((W & ~im) | iw) & inwin;
      I &= ~im & inwin;
      S_ &= ~im & inwin;
      CS &= ~im & inwin;
      D = ((D & ~im) | id) & inwin;
    }
    const bool wbad = __any(bad);
    STAMP(3);
    wsync();
    stage2();  // (rp is free after the exception pass: the next window's bytes fly behind the rest)
    // ---- 2: units -----------------------------------------------------------
    uint32_t U, SBm;
    int ub, sbb, n, nstarts;
    {
      SBm = L.sb[lane];
      const uint32_t carry = wave_shr1(W) >> 31;
      const uint32_t pw = (W << 1) | (lane ? carry : 0u);
      U = CS & (I | (W & (~pw | SBm)));
      L.brk[lane] = U | (S_ & CS) | SBm;
      L.um[lane] = U;
      L.dm[lane] = D;
      const uint32_t v = (uint32_t)__popc(U) | ((uint32_t)__popc(SBm) << 16);
      const uint32_t x = wave_incl_add(v);
      const uint32_t tot = lane_get(x, 63);
      const uint32_t ex = x - v;
      ub = (int)(ex & 0xFFFFu);
      sbb = (int)(ex >> 16);
      n = (int)(tot & 0xFFFFu);
      nstarts = (int)(tot >> 16);
      L.xm[256 + lane] = (uint32_t)ub;
    }
    // every sentence start distinct (no empty sentence shares one): a unit's
    // sentence is the number of starts at or before it, minus one
    const bool starts_distinct = nstarts == ns;
    // the first break / dirty byte in a later lane (a unit's span end and its
    // dirtiness come from the lane's own masks and these two positions,
    // instead of a search of the LDS masks per unit)
    int nxt_brk, nxt_dirty;
    {
      const uint32_t brk = U | (S_ & CS) | SBm;
      const uint64_t later = lane < 63 ? ~0ull << (lane + 1) : 0ull;
      const uint64_t mb = __ballot(brk != 0) & later, md = __ballot(D != 0) & later;
      wsync();  // (L.brk / L.dm of every lane written)
      nxt_brk = nb;
      nxt_dirty = CAP;
      if (mb) {
        const int j = __ffsll((unsigned long long)mb) - 1;
        nxt_brk = min(j * 32 + __ffs(L.brk[j]) - 1, nb);
      }
      if (md) {
        const int j = __ffsll((unsigned long long)md) - 1;
        nxt_dirty = j * 32 + __ffs(L.dm[j]) - 1;
      }
      L.xm[128 + lane] = lx_make(nxt_brk, nxt_dirty, sbb);
      // each sentence's first unit (units before its start: the owning lane's
      // base + its unit bits below the start) and its entry base; a unit's
      // entry is its rank in its sentence (an empty unit leaves a hole)
      if (lane <= ns) {
        const int pos = lane < ns ? (int)L.sst[lane] : nb;
        int uf = n;
        if (pos < nb) uf = (int)L.xm[256 + (pos >> 5)] + __popc(L.um[pos >> 5] & ((1u << (pos & 31)) - 1u));
        L.ufirst[lane] = (uint16_t)uf;
        if (lane < ns) L.ebs[lane] = (uint16_t)(pos - uf);
      }
    }
    STAMP(4);
    if (wbad) {
      fallback();
      return;
    }
    const int64_t obase = (A - base) - aoff;  // output index of window position 0
    const int64_t ent0 = obase - ebase;       // entry index of window position 0
    bool ovf = false;
    tbase = cur;  // the tile's first record slot (it moves with a chunk switch)
    tsl = 0;      // record slots the tile took so far
    for (int rb = 0; rb < n; rb += UCAP) {
      const int nr = min(UCAP, n - rb);
      if (lane == 0) L.misc[0] = 0;
      {
        // the round's unit start positions in unit order (each lane its own
        // bits: the loop runs the wave's largest count at about half the
        // lanes busy, so a unit's span end, dirtiness and sentence are
        // derived in the unit step below, one unit per lane)
        // Four units per iteration, every write unconditional: a rank outside
        // the round ([k0, k1) are the lane's units in it) writes a spare LDS
        // word instead (only the lane the round starts in skips any)
        uint16_t* const up = reinterpret_cast<uint16_t*>(L.xm);
        uint16_t* const spare = reinterpret_cast<uint16_t*>(&L.misc[3]);
        const uint32_t Ul = L.um[lane];
        const int p0 = lane * 32;
        const int k0 = max(rb - ub, 0), k1 = min(rb + nr - ub, (int)__popc(Ul));
        uint32_t m = Ul;
        for (int k = 0; k < k1; k += 4) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int kk = k + j;
            uint16_t* const dst = kk >= k0 && kk < k1 ? up + (ub + kk - rb) : spare;
            *dst = (uint16_t)(p0 + __builtin_ctz(m | 0x80000000u));
            m &= m - 1;
          }
        }
      }
      wsync();
      STAMP(5);
      // ---- 3, fast steps: 64 units per step (one per lane), in unit order.
      //      A clean unit of <= 24 bytes (no filler / expansion byte, not a
      //      literal special) loads its key from the window, hashes it and
      //      probes slot 0 of its home bucket (one 32-B load, an xor / or
      //      compare); a hit writes its entry (the vocab id at the unit's rank
      //      in its sentence, ebs).  Every other unit -- a probe miss, a dirty
      //      span, a special, a key longer than 24 bytes -- is listed for the
      //      record pass (its unit index, flagged MISS when the probe already
      //      missed).  The fast step holds no per-mode code: one path, no LDS
      //      writes but the list.
      // ---- 4, record pass over the listed units, 64 per step, in unit order:
      //      dirty words normalised, specials, > 100-char words -> [UNK], the
      //      probe of a dirty word, then the entries and, for a word no probe
      //      resolved, its WordPiece record from the key in registers.  Record
      //      slots are tile-relative, in unit order, from two ballots (a
      //      sentence's slots are then contiguous and its first is the
      //      exclusive sum of the earlier sentences' at the end).
      {
        const int mb0 = (int)P.maxb[0];
        const uint32_t vmask = P.vt_mask;
        const int mbf = min(mb0, FKEY);  // (a clean key of FKEY < len <= 24 bytes: probed in the record pass)
        // the unit: start p (window position), span end q = the next break
        // (the owning lane's own bits, else its later-lane position), dirty
        // (a filler / expansion byte in [p, q)) and sentence sj
        auto decode = [&](int u, bool valid, int& p, int& q, bool& dirty, uint32_t& sj) {
          p = valid ? (int)reinterpret_cast<const uint16_t*>(L.xm)[u] : 0;
          const int wl = p >> 5, b = p & 31, p0 = p & ~31;
          const uint32_t brk = L.brk[wl], Dl = L.dm[wl], SBl = L.sb[wl], lx = L.xm[128 + wl];
          const uint32_t rest = brk & ~((2u << b) - 1u);
          q = rest ? min(p0 + __ffs(rest) - 1, nb) : (int)(lx & 0xFFFu);
          uint32_t own = Dl & ~((1u << b) - 1u);
          if (q < p0 + 32) own &= (1u << (q - p0)) - 1u;
          dirty = valid && (own != 0 || (q > p0 + 32 && (int)((lx >> 12) & 0xFFFu) < q));
          if (starts_distinct) {
            sj = (lx >> 24) + (uint32_t)__popc(SBl & ((2u << b) - 1u)) - 1u;
          } else {
            int lo = 0, hi = ns - 1;  // last sentence starting at or before p
            while (lo < hi) {
              const int mid = (lo + hi + 1) >> 1;
              if ((int)L.sst[mid] <= p) lo = mid;
              else hi = mid - 1;
            }
            sj = (uint32_t)lo;
          }
        };
        // the deferred units of the round (u16: unit | MISS << 15), in the
        // lanes' unit bases' place (free once the sentences' first units are set)
        uint16_t* const dl = reinterpret_cast<uint16_t*>(L.xm + 192);
        constexpr uint32_t DL_MISS = 0x8000u;
        uint32_t ndef = 0;
        // FK steps per batch: every step's key, hash and probe loads first,
        // then the compares, so the batch's probe round trips overlap (the
        // loads of a batch are issued back to back; no store sits between
        // them and their first use)
        const bool fprobe = P.st == nullptr || LDDL_PROBE_L2;  // (the two-choice scan table: probed in the record pass)
        // (the entry buffer's last element: no unit's entry, no serial-path id reaches it,
        // capi.hip sizes it seg_tiles * 1 KiB + max_tok + 4096)
        const int64_t ent_spare = S.seg_tiles * 1024 + max_tok + 4095;
        for (int r = 0; r < nr; r += 64 * FK) {
          Key6 key[FK];
          uint4 fa[FK], fb[FK];
          bool probe[FK], dirty[FK];
          int len[FK];
          uint32_t sj[FK];
#pragma unroll
          for (int k = 0; k < FK; ++k) {
            const int u = r + 64 * k + lane;
            const bool valid = u < nr;
            int p, q;
            decode(u, valid, p, q, dirty[k], sj[k]);
            len[k] = q - p;
            probe[k] = fprobe && valid && !dirty[k] && len[k] <= mbf;
            // (every lane: the key's reads depend on p alone and fly with the mask reads)
            key[k] = FKEY == 16 ? load_key16(L.nb, p, len[k]) : load_key(L.nb, p, len[k]);
            probe[k] = probe[k] && !((key[k].d0 & 0xFFu) >= BS && (key[k].d0 & 0xFFu) < BS + 5);
            // (every lane loads: a lane with nothing to probe reads bucket 0)
            const uint32_t hk = probe[k] ? key_hash(key[k], len[k], 0u) : 0u;
            const uint4* bk = P.vt + 4 * (hk & vmask & ((LDDL_PROBE_L2 == 1 || LDDL_PROBE_L2 == 2) ? 0x3FFFu : ~0u));
            fa[k] = bk[0];
            fb[k] = bk[1];
          }
          STAMP(12);
#pragma unroll
          for (int k = 0; k < FK; ++k) {
            const int u = r + 64 * k + lane;
            const bool valid = u < nr;
            const uint32_t want = ((uint32_t)len[k] << 16) | 0x80000000u;
            // (branch-free: a branch around the compare leaves the batch's loads
            // pending on one path, and the join then waits for every store too)
            const bool eq = LDDL_PROBE_L2 >= 2 || slot_eq(fa[k], fb[k], key[k], want);
            const bool hit = probe[k] & eq;
            const uint32_t id = fb[k].z & 0xFFFFu;
            // every lane stores (no branch around a store: the join after one
            // waits for it): a hit its id, a deferred unit a hole the record
            // pass overwrites (same wave, same address, in order), a lane past
            // the round's units the segment buffer's spare last entry
            S.ent[valid ? ent0 + (int)L.ebs[sj[k]] + rb + u : ent_spare] = (uint16_t)(hit ? id : SPLIT_EHOLE);
            // ([CLS] / [SEP] come only from literal specials, never from WordPiece;
            // a flag past the sentence's max_tok cut is harmless: the masked
            // packer then checks the ids themselves)
            const bool spc = hit && (id == P.special[2] || id == P.special[3]);
            if (__ballot(spc) != 0 && spc) atomicOr(&L.sspec[sj[k] >> 5], 1u << (sj[k] & 31));
            // (a clean key longer than any whole-word key misses without a probe)
            const bool dfr = valid && !hit;
            const uint64_t D = __ballot(dfr);
            if (dfr)
              dl[ndef + lane_rank(D)] =
                  (uint16_t)((uint32_t)u | (!dirty[k] && len[k] <= 24 && (probe[k] || len[k] > mb0) ? DL_MISS : 0u));
            ndef += (uint32_t)__popcll(D);
          }
          STAMP(7);
        }
        wsync();
        for (int r = 0; r < (int)ndef; r += 64) {
          const bool valid = r + lane < (int)ndef;
          const uint32_t de = valid ? dl[r + lane] : 0u;
          const int u = (int)(de & 0x7FFFu);
          const bool miss = (de & DL_MISS) != 0;
          uint32_t w = 0;
          uint16_t id = U_EMPTY;
          int p, q;
          bool dirty;
          uint32_t sj;
          decode(u, valid, p, q, dirty, sj);
          STAMP(12);
          int src = p, len = valid ? q - p : 0;
          bool lovf = false;  // the tile falls back: side buffer full, or a queued word too long for a record
          if (dirty) {
            len = dirty_normalize(L, P, src, src + len, &src);
            lovf = len < 0;
            len = max(len, 0);
          }
          STAMP(13);
          Key6 key = {0, 0, 0, 0, 0, 0};
          if (len > 0 && len <= 24) key = load_key(L.nb, src, len);
          if (len > 0) {
            const uint32_t b0 = key.d0 & 0xFFu;
            if (!dirty && len <= 24 && b0 >= BS && b0 < BS + 5) {
              id = (uint16_t)P.special[b0 - BS];
            } else if (len > 100 && count_chars(L.nb, src, len) > 100) {
              id = (uint16_t)P.unk;
            } else {
              id = U_DEFER;
              w = 1;
              lovf |= len > KEYMAX;
            }
          }
          STAMP(6);
          if (w != 0 && !miss && len <= 24 && len <= mb0) {
            const uint32_t hk = key_hash(key, len, 0u), want = ((uint32_t)len << 16) | 0x80000000u;
            if (P.st && !LDDL_PROBE_L2) {
              // the scan table: both candidate slots loaded before either compare
              const uint4* s1 = P.st + 2 * (hk & P.st_mask);
              const uint4* s2 = P.st + 2 * (st_second(hk) & P.st_mask);
              const uint4 fa = s1[0], fb = s1[1], ga = s2[0], gb = s2[1];
              const bool h1 = slot_eq(fa, fb, key, want), h2 = slot_eq(ga, gb, key, want);
              if (h1 || h2) {
                id = (uint16_t)((h1 ? fb.z : gb.z) & 0xFFFFu);
                w = 0;
              }
            } else {
              const uint4* bk = P.vt + 4 * (hk & vmask & ((LDDL_PROBE_L2 == 1 || LDDL_PROBE_L2 == 2) ? 0x3FFFu : ~0u));
              const uint4 fa = bk[0], fb = bk[1];
              if (LDDL_PROBE_L2 >= 2 || slot_eq(fa, fb, key, want)) {
                id = (uint16_t)(fb.z & 0xFFFFu);
                w = 0;
              }
            }
          }
          if (__any(lovf)) {
            ovf = true;
            break;
          }
          STAMP(7);
          // ---- entries and records ----------------------------------------
          const uint32_t nsl = (valid && id == U_DEFER) ? (len <= KEY1 ? 1u : 2u) : 0u;
          const uint64_t N1 = __ballot(nsl != 0), N2 = __ballot(nsl == 2);
          const uint32_t need = (uint32_t)(__popcll(N1) + __popcll(N2));
          // this step's slots come from the wave's chunk; the tile's slots stay
          // contiguous: on a chunk switch, the ones it took in earlier steps
          // move to the new chunk (entries hold tile-relative slots)
          if (need > 0 && cur + need > cend) {
            if (tsl + need > SPLIT_CHUNK) {  // (a tile with > 1024 slots)
              ovf = true;
              break;
            }
            if (chunk >= 0 && lane == 0) S.chunk_fill[chunk] = tbase - cbase;  // (the moved ones not run)
            int c = 0;
            if (lane == 0) c = (int)atomicAdd(S.chunk_ctr, 1u);
            c = __builtin_amdgcn_readfirstlane(c);
            if ((uint32_t)c >= S.n_chunks) {  // record capacity exhausted
              chunk = -1;
              cur = cend = cbase = tbase = 0;
              ovf = true;
              break;
            }
            chunk = c;
            cbase = (uint32_t)c * SPLIT_CHUNK;
            cend = cbase + SPLIT_CHUNK;
            if (tsl) {
              // (records this wave stored in an earlier step: drain its stores first)
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
              for (int k = 0; k < 4; ++k)
                for (uint32_t i = lane; i < tsl; i += 64) *recq(S, k, cbase + i) = *recq(S, k, tbase + i);
              // (piece counts: wp_kernel writes the moved words' own; the moved
              // extension slots count 0)
              for (uint32_t i = lane; i < tsl; i += 64) S.cnt8[cbase + i] = 0;
            }
            tbase = cbase;
            cur = cbase + tsl;
          }
          STAMP(10);
          const uint32_t o = tsl + (uint32_t)(lane_rank(N1) + lane_rank(N2));  // tile-relative slot
          if (valid) {
            S.ent[ent0 + (int)L.ebs[sj] + rb + u] =
                (uint16_t)(id == U_EMPTY ? SPLIT_EHOLE : id != U_DEFER ? id : (SPLIT_EDEF | o));
            if (id == U_EMPTY || id == U_DEFER) atomicAdd(&L.sacc[sj], nsl | 0x10000u);
            // ([CLS] / [SEP] come only from literal specials, never from WordPiece;
            // a flag past the sentence's max_tok cut is harmless: the masked
            // packer then checks the ids themselves)
            else if (id == P.special[2] || id == P.special[3]) atomicOr(&L.sspec[sj >> 5], 1u << (sj & 31));
          }
          if (nsl) {
            // the record {len | slots << 8 | valid, count, key bytes 0..55}
            const uint32_t slot = tbase + o;
            uint32_t kd[6] = {key.d0, key.d1, key.d2, key.d3, key.d4, key.d5};
            const int a = src >> 2;
            const uint32_t sh = (uint32_t)(src & 3);
            if (len > 24) {
              uint32_t xx[7];
#pragma unroll
              for (int i = 0; i < 7; ++i) xx[i] = L.nb[a + i];
#pragma unroll
              for (int i = 0; i < 6; ++i) kd[i] = __builtin_amdgcn_alignbyte(xx[i + 1], xx[i], sh);
            }
            if (LDDL_PROBE_REC < 2) *recq(S, 0, slot) = make_uint4((uint32_t)len | (nsl << 8) | 0x80000000u, 0u, kd[0], kd[1]);
            if (LDDL_PROBE_REC < 1) *recq(S, 1, slot) = make_uint4(kd[2], kd[3], kd[4], kd[5]);
            // key bytes 24..55 (wp_kernel reads them only for a longer key)
            if (LDDL_PROBE_REC < 1 && len > 24) {
              uint32_t xx[9];
#pragma unroll
              for (int i = 0; i < 9; ++i) xx[i] = L.nb[a + 6 + i];
              uint32_t kq[8];
#pragma unroll
              for (int i = 0; i < 8; ++i) kq[i] = keep_bytes(__builtin_amdgcn_alignbyte(xx[i + 1], xx[i], sh), len - 24 - 4 * i);
              *recq(S, 2, slot) = make_uint4(kq[0], kq[1], kq[2], kq[3]);
              *recq(S, 3, slot) = make_uint4(kq[4], kq[5], kq[6], kq[7]);
            }
            if (nsl == 2) {  // the extension slot: a zero header (skipped by wp_kernel)
              *recq(S, 0, slot + 1) = make_uint4(0, 0, 0, 0);
              S.cnt8[slot + 1] = 0;  // (its pieces buffer holds pieces 28.. of the word)
            }
          }
          tsl += need;
          cur += need;
          wsync();
          STAMP(8);
        }
      }
      if (ovf) break;
    }  // rounds
    if (ovf) {
      fallback();
      return;
    }
    {
      // one 8-B record per sentence for expand / count: entries (units, holes
      // included) | its first slot relative to the tile's << 16, the tile's
      // first slot; the direct ids so far (count_kernel adds the pieces)
      const uint32_t acc = lane < ns ? L.sacc[lane] : 0u;
      const uint32_t nsl = acc & 0xFFFFu;
      const uint32_t sq0 = wave_incl_add(nsl) - nsl;
      if (lane < ns) {
        const int64_t s = sa + lane_here();
        const uint32_t ne = (uint32_t)L.ufirst[lane + 1] - (uint32_t)L.ufirst[lane];
        S.smeta[s] = make_uint2(ne | (sq0 << 16), tbase);
        S.snslot[s] = (uint16_t)nsl;
        P.out_ntok[s] = (int)(ne - (acc >> 16));
        if (P.sent_spec) P.sent_spec[s] = (uint8_t)((L.sspec[lane >> 5] >> (lane & 31)) & 1u);
      }
    }
  
    }();
    STAMP(9);
    if (DBG) acc[11] += 1;
  }
  if (DBG && lane == 0)
    for (int k = 0; k < 12; ++k) atomicAdd((unsigned long long*)&P.dbg[k], (unsigned long long)acc[k]);
  if (DBG && lane == 0)
    for (int k = 12; k < 17; ++k) atomicAdd((unsigned long long*)&P.dbg[6 + k], (unsigned long long)acc[k]);
#undef STAMP
  if (chunk >= 0 && lane == 0) S.chunk_fill[chunk] = cur - cbase;
}

// ------------------------------------------------------------ WordPiece --
constexpr int KB_DW = 16;  // per-lane key buffer in LDS: dword i of lane l at [i][l] (conflict-free
                           // reads at any per-lane offset); reads past dword 15 are clamped (zeros)

// u16 index of piece q in a record (slot 0: pieces 0..27 from byte 8; the
// extension slot keeps its zero header: pieces 28.. from its byte 4)
__device__ __forceinline__ int piece_at(int q) { return q < 28 ? 4 + q : 34 + (q - 28); }

template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void wp_kernel(TokParams P, SplitParams S) {
  __shared__ uint32_t bloom[BLOOM_WORDS];
  __shared__ uint32_t kbuf[WAVES * 64 * KB_DW];
  for (int i = threadIdx.x; i < BLOOM_WORDS; i += 64 * WAVES) bloom[i] = P.vbloom[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* kb = kbuf + wv * 64 * KB_DW + lane;  // dword i at kb[64 * i]
  auto kdw = [&](int i) { return kb[64 * min(i, KB_DW - 1)]; };
  auto kbyte = [&](int i) { return (kdw(i >> 2) >> (8 * (i & 3))) & 0xFFu; };
  const uint32_t nch = min(__builtin_amdgcn_readfirstlane(*S.chunk_ctr), S.n_chunks);
  const uint32_t nwaves = gridDim.x * WAVES;
  const int mb0 = (int)P.maxb[0], mb1 = (int)P.maxb[1];
  const uint32_t vmask = P.vt_mask;
  // the wave's slot stream: unit gw first, then units handed out by a
  // counter (chunks hold different work: dynamic hand-out balances the
  // launch's tail); a unit is half a chunk's filled slots (the launch's
  // last units are shorter); the next unit is fetched one unit ahead, so
  // the atomic's round trip flies with the current unit's loads.  (A record
  // and its extension slot may fall in different halves: the extension
  // slot's zero header is skipped wherever it is.)
  uint32_t* const wctr = S.chunk_ctr + 1;  // zeroed with chunk_ctr per segment
  const uint32_t nun = 2 * nch;
  uint32_t u = blockIdx.x * WAVES + wv, c = u >> 1, off = 0, fill = 0;
  uint32_t cn = 0;  // (lane 0) the next unit
  auto take = [&]() {  // unit u: slots [off, fill) of chunk c
    const uint32_t f = __builtin_amdgcn_readfirstlane(S.chunk_fill[c]);
    off = (u & 1u) ? f >> 1 : 0u;
    fill = (u & 1u) ? f : f >> 1;
  };
  if (u < nun) {
    take();
    if (lane == 0) cn = nwaves + atomicAdd(wctr, 1u);
  }
  auto advance = [&]() {
    while (off >= fill && u < nun) {
      u = (uint32_t)__builtin_amdgcn_readlane((int)cn, 0);
      c = u >> 1;
      off = 0;
      fill = 0u;
      if (u < nun) {
        take();
        if (lane == 0) cn = nwaves + atomicAdd(wctr, 1u);
      }
    }
  };
  advance();
  uint32_t nrec = 0;  // records this lane ran
  int r = -1;    // record slot being tokenised
  int pr = -1;   // record slot loaded, not begun
  uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0, q2 = q0, q3 = q0;
  bool qlong = false;  // q2 / q3 of the pending record loaded
  int s = 0, we = 0, e = 0, np = 0, bslot = -1;
  uint32_t cont = 0;
  bool asc = false;
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0;
  uint32_t H0 = VSEED, H1 = 0, H2 = 0, H3 = 0, H4 = 0, H5 = 0, H6 = 0;
  auto load_cand = [&]() {
    const int a = s >> 2;
    const uint32_t sh = (uint32_t)(s & 3);
    const uint32_t x0 = kdw(a), x1 = kdw(a + 1), x2 = kdw(a + 2), x3 = kdw(a + 3), x4 = kdw(a + 4), x5 = kdw(a + 5),
                   x6 = kdw(a + 6);
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
  auto selH = [&](int q) { return q <= 0 ? H0 : q == 1 ? H1 : q == 2 ? H2 : q == 3 ? H3 : q == 4 ? H4 : q == 5 ? H5 : H6; };
  auto selD = [&](int q) { return q <= 0 ? c0 : q == 1 ? c1 : q == 2 ? c2 : q == 3 ? c3 : q == 4 ? c4 : c5; };
  auto hash_len = [&](int l) {  // == vhash of the candidate [s, s+l)
    const uint32_t h = l >= 12 ? H3 : vmix(vmix(vmix(VSEED, vmask_rem(c0, l)), vmask_rem(c1, l - 4)), vmask_rem(c2, l - 8));
    return vfinal(h, (uint32_t)l, cont);
  };
  auto bkey_len = [&](int l) {  // == vbkey of the candidate [s, s+l)
    const int lc = min(l, 24), q = lc >> 2, rr = lc & 3;
    return vbkey(selH(q), rr ? selD(q) & ((1u << (8 * rr)) - 1u) : 0u, (uint32_t)l, cont);
  };
  auto bloom_ok = [&](uint32_t h) {
    const uint32_t bb = vbloom_bits(h);
    return (bloom[vbloom_word(h)] & bb) == bb;
  };
  auto shrink = [&]() {  // previous char boundary
    --e;
    if (!(asc && e - s < 24))
      while (e > s && (kbyte(e) & 0xC0u) == 0x80u) --e;
  };
  auto start_piece = [&](int maxb) {
    bslot = -1;
    load_cand();
    e = min(we, s + maxb);
    if (e < we && !(asc && e - s < 24))
      while (e > s && (kbyte(e) & 0xC0u) == 0x80u) --e;
  };
  // (the pieces and count go to a buffer of their own, so the
  // record lines other lanes are still loading stay read-only)
  uint4* const outs = S.pcs;
  auto rec16 = [&]() { return reinterpret_cast<uint16_t*>(outs + (size_t)r * 4); };
  // pieces 0-3 (nearly every word's all) held in two registers and stored
  // with the count as the slot's dense 16-B head at the end (what expand loads)
  uint32_t pw01 = 0, pw23 = 0;
  auto put_piece = [&](int k, uint32_t id) {
    if (k < 4) {
      const uint32_t sh = 16u * (uint32_t)(k & 1);
      const uint32_t keep = ~(0xFFFFu << sh), val = id << sh;
      if (k < 2) pw01 = (pw01 & keep) | val;
      else pw23 = (pw23 & keep) | val;
    } else {
      rec16()[piece_at(k)] = (uint16_t)id;
    }
  };
  auto finish = [&]() {
    S.pch[r] = make_uint4((uint32_t)np, pw01, pw23, 0u);
    S.cnt8[r] = (uint8_t)np;
    r = -1;
  };
  // optional stamps (P.dbg, LDDL_TOK_DEBUG=1): A (Bloom scan + bucket
  // issue), B (refill issue), C (compare; waits for the loads), D (record
  // start), steps, lane-steps with a record
  uint64_t wacc[6] = {0, 0, 0, 0, 0, 0}, wprev = 0;
  const bool wdbg = P.dbg != nullptr;
#define WP_STAMP(k)                                                              \
  if (wdbg) {                                                                    \
    uint64_t t_;                                                                 \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    wacc[k] += t_ - wprev;                                                       \
    wprev = t_;                                                                  \
  }
  if (wdbg) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(wprev)::"memory");
  for (;;) {
    // ---- A: candidate of each working lane: the longest length the Bloom
    //      filter does not rule out, then its bucket load
    bool fail = false;
    uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0, b0 = a0, b1 = a0;
    if (r >= 0) {
      if (bslot < 0) {
        int len = e - s;
        bool found = false;
        uint32_t hcur = 0;
        // candidates of <= 24 bytes: the dword-group Bloom scan over every
        // byte length (a non-ASCII prefix ending inside a character never
        // equals a vocab key, which is valid UTF-8: its Bloom false
        // positives only cost a failed probe, then shrink() steps back to a
        // character boundary)
        if (len <= 24) {
          int fl = 0;
          int ga = 0;
#define TOK5_EXT(j, Hj1) \
  ga = ((ga == (j)) & (4 * ((j) + 1) < len) & bloom_ok(vbkey_ext(Hj1, 4 * ((j) + 1), cont))) ? (j) + 1 : ga;
          TOK5_EXT(0, H1)
          TOK5_EXT(1, H2)
          TOK5_EXT(2, H3)
          TOK5_EXT(3, H4)
          TOK5_EXT(4, H5)
#undef TOK5_EXT
#define TOK5_GROUP(k, Hk, Hk1, ck)                                                                              \
  if (fl == 0 && 4 * (k) < len && (k) <= ga) {                                                                  \
    const uint32_t g4 = vbkey(Hk1, 0u, 4 * (k) + 4, cont), g3 = vbkey(Hk, (ck) & 0xFFFFFFu, 4 * (k) + 3, cont), \
                   g2 = vbkey(Hk, (ck) & 0xFFFFu, 4 * (k) + 2, cont),                                           \
                   g1 = vbkey(Hk, (ck) & 0xFFu, 4 * (k) + 1, cont);                                             \
    const bool o4 = (4 * (k) + 4 <= len) & bloom_ok(g4), o3 = (4 * (k) + 3 <= len) & bloom_ok(g3),              \
               o2 = (4 * (k) + 2 <= len) & bloom_ok(g2), o1 = bloom_ok(g1);                                     \
    if (o4 | o3 | o2 | o1) fl = o4 ? 4 * (k) + 4 : o3 ? 4 * (k) + 3 : o2 ? 4 * (k) + 2 : 4 * (k) + 1;           \
  }
          TOK5_GROUP(5, H5, H6, c5)
          TOK5_GROUP(4, H4, H5, c4)
          TOK5_GROUP(3, H3, H4, c3)
          TOK5_GROUP(2, H2, H3, c2)
          TOK5_GROUP(1, H1, H2, c1)
          TOK5_GROUP(0, H0, H1, c0)
#undef TOK5_GROUP
          found = fl > 0;
          e = s + fl;
          if (found) hcur = hash_len(fl);
        } else {
          while (e > s) {
            if (bloom_ok(bkey_len(e - s))) {
              hcur = hash_len(e - s);
              found = true;
              break;
            }
            shrink();
          }
        }
        if (found) bslot = (int)(hcur & vmask);
        else fail = true;
      }
      if (!fail) {
        const uint4* bk = P.vt + 4 * (uint32_t)bslot;
        a0 = bk[0];
        a1 = bk[1];
        b0 = bk[2];
        b1 = bk[3];
      }
    }
    WP_STAMP(0)
    // ---- B: lanes without a loaded record take the next slots of the
    //      stream, working lanes included (one record ahead: a lane that
    //      finishes its word in C begins the next one in D of the same step
    //      instead of idling a step); their loads fly with the bucket loads
    {
      const uint64_t idle = __ballot(pr < 0);
      if (idle != 0 && u < nun) {
        const uint32_t avail = fill - off;
        const int k = lane_rank(idle);
        if (pr < 0 && (uint32_t)k < avail) {
          pr = (int)(c * SPLIT_CHUNK + off + (uint32_t)k);
          q0 = *recq(S, 0, (uint32_t)pr);
          q1 = *recq(S, 1, (uint32_t)pr);
          // key bytes 24.. only for a longer key: loaded at its start (the
          // record begins a step later); a key of <= 24 bytes is zero past them
          q2 = q3 = make_uint4(0, 0, 0, 0);
          qlong = false;
        }
        off += min((uint32_t)__popcll(idle), avail);
        advance();
      }
    }
    WP_STAMP(1)
    // ---- C: compare and advance
    if (r >= 0) {
      if (fail) {  // some position has no match: the whole word is [UNK]
        np = 0;
        put_piece(0, (uint32_t)P.unk);
        np = 1;
        finish();
      } else {
        const int len = e - s;
        const int lc = min(len, 24);
        auto msk = [&](int k, uint32_t cc) {  // the key's bytes of dword k, branch-free
          const int nbk = min(max(lc - 4 * k, 0), 4);
          return cc & (nbk >= 4 ? 0xFFFFFFFFu : ((1u << (8 * nbk)) - 1u));
        };
        const uint32_t m0c = msk(0, c0), m1c = msk(1, c1), m2c = msk(2, c2), m3c = msk(3, c3), m4c = msk(4, c4),
                       m5c = msk(5, c5);
        const uint32_t want = ((uint32_t)len << 16) | (cont << 24) | 0x80000000u;
        bool m0 = (((a1.z & 0xFFFF0000u) ^ want) | (a0.x ^ m0c) | (a0.y ^ m1c) | (a0.z ^ m2c) | (a0.w ^ m3c) |
                   (a1.x ^ m4c) | (a1.y ^ m5c)) == 0u;
        bool m1 = (((b1.z & 0xFFFF0000u) ^ want) | (b0.x ^ m0c) | (b0.y ^ m1c) | (b0.z ^ m2c) | (b0.w ^ m3c) |
                   (b1.x ^ m4c) | (b1.y ^ m5c)) == 0u;
        if (len > 24) {  // the rest of a long key against the pool
          if (m0)
            for (int k = 24; k < len; ++k) m0 = m0 && kbyte(s + k) == P.pool[a1.w + k];
          if (m1)
            for (int k = 24; k < len; ++k) m1 = m1 && kbyte(s + k) == P.pool[b1.w + k];
        }
        if (m0 || m1) {
          put_piece(np, (m0 ? a1.z : b1.z) & 0xFFFFu);
          ++np;
          s = e;
          if (s >= we) {
            finish();
          } else {
            cont = 1;
            start_piece(mb1);
          }
        } else if (!(a1.z & 0x80000000u) || !(b1.z & 0x80000000u)) {
          bslot = -1;  // an empty slot ends the probe sequence: no such key
          shrink();
        } else {
          bslot = (int)(((uint32_t)bslot + 1u) & vmask);
        }
      }
    }
    WP_STAMP(2)
    // ---- D: an extension slot is dropped (refilled in the next B), a long
    //      key's bytes 24.. are loaded (working lanes too: ready when their
    //      word ends), idle lanes with a loaded record begin it
    if (pr >= 0) {
      if (q0.x == 0u) {  // an extension slot
        pr = -1;
      } else if ((q0.x & 0xFFu) > 24u && !qlong) {
        q2 = *recq(S, 2, (uint32_t)pr);
        q3 = *recq(S, 3, (uint32_t)pr);
        qlong = true;
      } else if (r < 0) {
        const int len = (int)(q0.x & 0xFFu);
        kb[0] = q0.z; kb[64] = q0.w;
        kb[128] = q1.x; kb[192] = q1.y; kb[256] = q1.z; kb[320] = q1.w;
        kb[384] = q2.x; kb[448] = q2.y; kb[512] = q2.z; kb[576] = q2.w;
        kb[640] = q3.x; kb[704] = q3.y; kb[768] = q3.z; kb[832] = q3.w;
        kb[896] = 0u;
        kb[960] = 0u;
        r = pr;
        pr = -1;
        ++nrec;
        s = 0;
        we = len;
        np = 0;
        cont = 0;
        start_piece(mb0);
      }
    }
    WP_STAMP(3)
    if (wdbg) {
      wacc[4] += 1;
      wacc[5] += __popcll(__ballot(r >= 0));
    }
    if (__ballot(r >= 0 || pr >= 0) == 0 && u >= nun) break;
  }
  if (wdbg && lane == 0)
    for (int k = 0; k < 6; ++k) atomicAdd((unsigned long long*)&P.dbg[12 + k], (unsigned long long)wacc[k]);
#undef WP_STAMP
  if (S.n_rec) {
    const uint32_t tot = lane_get(wave_incl_add(nrec), 63);
    if (lane == 0 && tot) atomicAdd(S.n_rec, (unsigned long long)tot);
  }
}

// ---------------------------------------------------- WordPiece by trie --
// The same records, pieces and counts as wp_kernel, found by walking the
// vocab's double-array trie (tok_tables.h build_trie, common.h trie_*): per
// step one byte of the key and one 8-B entry load; the walk from a piece
// start ends where no key extends the bytes read, and the longest prefix it
// accepted on the way is the piece (greedy longest-match-first, exactly
// WordPiece's); the next piece's walk starts from the "##" root at its end.
// No Bloom filter and no key hashing: ~30 instructions per step against
// ~470 per step of wp_kernel's Bloom scan.  One record per lane with refill,
// as wp_kernel (a lane whose word ends begins the next record in the same
// step); WPT_STEPS steps per round of the refill bookkeeping.
// Measured, not kept as the default (LDDL_WP_ALGO=trie selects it):
// 2.08 / 2.34 / 2.56 ms per GB of corpus at WPT_STEPS 8 / 4 / 2 against
// wp_kernel's 1.28 (profiles/r5_wp_trie_ab.txt).  The steps are cheap but
// each is a dependent ~L2 round trip (~13 per record), and the refill
// bookkeeping per round costs what the Bloom scan saves.
#ifdef LDDL_WPT_STEPS
constexpr int WPT_STEPS = LDDL_WPT_STEPS;  // (A/B builds, tools/ab_build.py)
#else
constexpr int WPT_STEPS = 8;
#endif

template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void wpt_kernel(TokParams P, SplitParams S) {
  __shared__ uint32_t kbuf[WAVES * 64 * KB_DW];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* kb = kbuf + wv * 64 * KB_DW + lane;  // dword i at kb[64 * i]
  auto kbyte = [&](int i) { return (kb[64 * min(i >> 2, KB_DW - 1)] >> (8 * (i & 3))) & 0xFFu; };
  const uint32_t nch = min(__builtin_amdgcn_readfirstlane(*S.chunk_ctr), S.n_chunks);
  const uint32_t nwaves = gridDim.x * WAVES;
  const uint2* const trie = P.trie;
  const uint32_t rb0 = P.trie_base[0], rb1 = P.trie_base[1];
  uint32_t* const wctr = S.chunk_ctr + 1;  // zeroed with chunk_ctr per segment
  uint32_t c = blockIdx.x * WAVES + wv, off = 0, fill = 0;
  uint32_t cn = 0;  // (lane 0) the next chunk
  if (c < nch) {
    fill = __builtin_amdgcn_readfirstlane(S.chunk_fill[c]);
    if (lane == 0) cn = nwaves + atomicAdd(wctr, 1u);
  }
  auto advance = [&]() {
    while (off >= fill && c < nch) {
      c = (uint32_t)__builtin_amdgcn_readlane((int)cn, 0);
      off = 0;
      fill = 0u;
      if (c < nch) {
        fill = __builtin_amdgcn_readfirstlane(S.chunk_fill[c]);
        if (lane == 0) cn = nwaves + atomicAdd(wctr, 1u);
      }
    }
  };
  advance();
  uint32_t nrec = 0;
  int r = -1;   // record slot being tokenised
  int pr = -1;  // record slot loaded, not begun
  uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0, q2 = q0, q3 = q0;
  bool qlong = false;
  int q = 0, len = 0, ps = 0, la = -1, np = 0;
  uint32_t node = 0, nbase = 0, laid = 0;
  uint4* const outs = S.pcs;
  uint32_t pw01 = 0, pw23 = 0;
  auto put_piece = [&](int k, uint32_t id) {
    if (k < 4) {
      const uint32_t sh = 16u * (uint32_t)(k & 1);
      const uint32_t keep = ~(0xFFFFu << sh), val = id << sh;
      if (k < 2) pw01 = (pw01 & keep) | val;
      else pw23 = (pw23 & keep) | val;
    } else {
      reinterpret_cast<uint16_t*>(outs + (size_t)r * 4)[piece_at(k)] = (uint16_t)id;
    }
  };
  auto finish = [&]() {
    S.pch[r] = make_uint4((uint32_t)np, pw01, pw23, 0u);
    S.cnt8[r] = (uint8_t)np;
    r = -1;
  };
  for (;;) {
    // ---- the walk: WPT_STEPS trie steps of each working lane
#pragma unroll
    for (int st = 0; st < WPT_STEPS; ++st) {
      if (r >= 0) {
        const uint32_t idx = nbase + kbyte(q);
        const uint2 t = trie[idx];
        if (trie_check(t) == node) {
          node = idx;
          nbase = trie_base(t);
          ++q;
          if (trie_accept(t)) {
            la = q;
            laid = trie_id(t);
          }
          if (q < len) continue;
        }
        // the walk stopped: at the word's end, or no key extends [ps, q]
        if (la >= 0) {
          put_piece(np, laid);
          ++np;
          if (la == len) {
            finish();
          } else {  // the next piece, "##", from the end of this one
            q = ps = la;
            la = -1;
            node = 1;
            nbase = rb1;
          }
        } else {  // some position has no match: the whole word is [UNK]
          np = 0;
          put_piece(0, (uint32_t)P.unk);
          np = 1;
          finish();
        }
      }
    }
    // ---- idle lanes take the next slots of the stream (one record ahead)
    {
      const uint64_t idle = __ballot(pr < 0);
      if (idle != 0 && c < nch) {
        const uint32_t avail = fill - off;
        const int k = lane_rank(idle);
        if (pr < 0 && (uint32_t)k < avail) {
          pr = (int)(c * SPLIT_CHUNK + off + (uint32_t)k);
          q0 = *recq(S, 0, (uint32_t)pr);
          q1 = *recq(S, 1, (uint32_t)pr);
          q2 = q3 = make_uint4(0, 0, 0, 0);
          qlong = false;
        }
        off += min((uint32_t)__popcll(idle), avail);
        advance();
      }
    }
    // ---- an extension slot is dropped, a long key's bytes 24.. loaded, idle
    //      lanes with a loaded record begin it
    if (pr >= 0) {
      if (q0.x == 0u) {
        pr = -1;
      } else if ((q0.x & 0xFFu) > 24u && !qlong) {
        q2 = *recq(S, 2, (uint32_t)pr);
        q3 = *recq(S, 3, (uint32_t)pr);
        qlong = true;
      } else if (r < 0) {
        len = (int)(q0.x & 0xFFu);
        kb[0] = q0.z; kb[64] = q0.w;
        kb[128] = q1.x; kb[192] = q1.y; kb[256] = q1.z; kb[320] = q1.w;
        kb[384] = q2.x; kb[448] = q2.y; kb[512] = q2.z; kb[576] = q2.w;
        kb[640] = q3.x; kb[704] = q3.y; kb[768] = q3.z; kb[832] = q3.w;
        kb[896] = 0u;
        kb[960] = 0u;
        r = pr;
        pr = -1;
        ++nrec;
        q = ps = 0;
        la = -1;
        np = 0;
        node = 0;
        nbase = rb0;
      }
    }
    if (__ballot(r >= 0 || pr >= 0) == 0 && c >= nch) break;
  }
  if (S.n_rec) {
    const uint32_t tot = lane_get(wave_incl_add(nrec), 63);
    if (lane == 0 && tot) atomicAdd(S.n_rec, (unsigned long long)tot);
  }
}

template <int WAVES>
static hipError_t launch_wpt(const TokParams& P, const SplitParams& S, int n_cu, hipStream_t s) {
  static int per_cu = 0;
  if (per_cu == 0 &&
      (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, wpt_kernel<WAVES>, 64 * WAVES, 0) != hipSuccess ||
       per_cu < 1))
    per_cu = 1;
  const int64_t grid = (int64_t)n_cu * per_cu;
  hipLaunchKernelGGL(wpt_kernel<WAVES>, dim3((unsigned)grid), dim3(64 * WAVES), 0, s, P, S);
  return hipGetLastError();
}

// ---------------------------------------------------------------- count --
// Final token count per sentence of the segment: its direct ids (the scan's
// entries that are vocab ids) + the pieces of its queued words (wp_kernel's
// per-slot counts over the sentence's contiguous record slots), capped at
// max_tok; a fallback tile's sentences keep the count the serial path wrote.
// (CNT_U sentences per thread per pass, 256 apart: each level of their
// chains -- metadata, then the slot counts -- loaded for all of them first)
constexpr int CNT_U = 4;
__global__ __launch_bounds__(256) void count_kernel(TokParams P, SplitParams S) {
  const int64_t sA = S.tile_sent[S.t0], sB = S.tile_sent[S.t1];
  const int64_t stride = (int64_t)gridDim.x * 256 * CNT_U;
  for (int64_t s0 = sA + (int64_t)blockIdx.x * 256 * CNT_U + threadIdx.x; s0 < sB; s0 += stride) {
    uint2 m[CNT_U];
    int32_t t[CNT_U];
    uint32_t n[CNT_U];
#pragma unroll
    for (int u = 0; u < CNT_U; ++u) {
      const int64_t s = s0 + 256 * u;
      const bool in = s < sB;
      m[u] = in ? S.smeta[s] : make_uint2(SPLIT_NENT_FB, 0u);
      t[u] = in ? P.out_ntok[s] : 0;
      n[u] = in ? S.snslot[s] : 0u;
    }
#pragma unroll
    for (int u = 0; u < CNT_U; ++u) {
      if ((m[u].x & 0xFFFFu) != SPLIT_NENT_FB) {
        const uint32_t q = m[u].y + (m[u].x >> 16);
        for (uint32_t k = 0; k < n[u]; ++k) t[u] += S.cnt8[q + k];
        t[u] = min(t[u], P.max_tok);
      }
    }
#pragma unroll
    for (int u = 0; u < CNT_U; ++u)
      if (s0 + 256 * u < sB) P.out_ntok[s0 + 256 * u] = t[u];
  }
}

// --------------------------------------------------------------- expand --
// Dense output: a wave per group of 64 sentences; their entries (a vocab id,
// a hole, or a queued word's record) in steps of 64, one per lane.  An entry's
// sentence: the group's non-empty sentences are numbered in order, each marks
// its first entry's lane in an LDS tag array (tagged by the step, so nothing
// is cleared), one ballot reads the marks back, and an entry's sentence is
// the marks at or below its lane (v_mbcnt) plus those of earlier steps; the
// step's entries are loaded one step ahead, so each
// step's record loads (count + first 4 pieces, one 12-B load) fly with the
// next step's entry loads.  A scan of the step's token counts, less its value
// at the sentence's first entry (one ds_bpermute), gives each token's position
// in its sentence, written at out_tok_off[s] + position while below the
// sentence's final count (count_kernel) and out_cap.
struct ExpSent {
  int64_t eb;    // entry index of the sentence's entry g (group numbering) = eb + g
  int64_t dst;   // output index of its first token
  uint32_t qb;   // the tile's first record slot
  uint32_t lim;  // tokens it writes: min(final count, out_cap - dst)
  uint32_t e0;   // its first entry (group numbering)
  uint32_t pad;
};
struct ExpLds {
  ExpSent sn[64];    // the group's non-empty sentences, in order
  uint32_t hf[64];   // hf[k] = the step's tag: some sentence's first entry is the step's entry k
};

__global__ __launch_bounds__(256) void expand_kernel(TokParams P, SplitParams S) {
  __shared__ ExpLds X[4];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  ExpLds& E = X[wv];
  const int64_t sA = uni64(S.tile_sent[S.t0]), sB = uni64(S.tile_sent[S.t1]);
  const int64_t base = P.sent_off[0], ebase = S.t0 << 10;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
  const uint4* const pcs = S.pcs;
  const uint4* const pch = S.pch;
  uint32_t tag = 0;  // per step, across the groups: hf needs no clearing
  E.hf[lane] = 0u;
  for (int64_t g0 = sA + ((int64_t)blockIdx.x * 4 + wv) * 64; g0 < sB; g0 += nwaves * 64) {
    const int64_t s = g0 + lane;
    uint32_t ne = 0;
    int64_t eoff = 0, d = 0;
    uint32_t qb = 0, lim = 0;
    if (s < sB) {
      const uint2 m = S.smeta[s];
      const int32_t nt = P.out_ntok[s];
      ne = m.x & 0xFFFFu;
      if (ne == SPLIT_NENT_FB) ne = (uint32_t)nt;  // the serial path's ids, all direct
      d = P.out_tok_off[s];
      eoff = P.sent_off[s] - base - ebase;
      qb = (m.x & 0xFFFFu) == SPLIT_NENT_FB ? 0u : m.y;
      lim = (uint32_t)max((int64_t)0, min((int64_t)nt, P.out_cap - d));
    }
    const uint32_t x = wave_incl_add(ne);
    const uint32_t e0 = x - ne;
    const uint32_t T = lane_get(x, 63);
    ExpSent es;
    es.eb = eoff - (int64_t)e0;
    es.dst = d;
    es.qb = qb;
    es.lim = lim;
    es.e0 = e0;
    es.pad = 0;
    const uint64_t nzm = __ballot(ne != 0);
    if (ne != 0) E.sn[bits_below(nzm)] = es;
    // the sentence (non-empty rank) of each entry of step st (entries st + lane)
    uint32_t hcar = 0;  // non-empty sentences that start before the step
    auto owner = [&](uint32_t st) -> uint32_t {
      ++tag;
      if (ne != 0 && e0 - st < 64u) E.hf[e0 - st] = tag;
      wsync();
      const bool head = E.hf[lane] == tag;
      const uint64_t hm = __ballot(head);
      const uint32_t o = hcar + (uint32_t)bits_below(hm) + (head ? 0u : (uint32_t)-1);
      hcar += (uint32_t)__popcll(hm);
      return o;
    };
    // EXP_K steps at a time, in three phases: the entry loads of all of them,
    // then their record loads, then their tokens -- every load of a phase in
    // flight together (the compiler drains the vector memory counter before
    // the first use of a load whenever stores are pending, so a pipeline
    // across loop iterations would wait at every step; here it waits twice
    // per EXP_K steps)
#ifndef LDDL_EXP_K
#define LDDL_EXP_K 5
#endif
    constexpr int EXP_K = LDDL_EXP_K;  // 5: 64 VGPRs, 8 waves per SIMD (6: 68 VGPRs, 7 waves; 8: 80, 6 waves)
    uint32_t carry = 0;
    for (uint32_t st0 = 0; st0 < T; st0 += 64 * EXP_K) {
      uint32_t xj[EXP_K], xv[EXP_K];
      bool xin[EXP_K];
#pragma unroll
      for (int k = 0; k < EXP_K; ++k) {
        const uint32_t st = st0 + 64 * k;
        xj[k] = 0;
        xv[k] = 0;
        xin[k] = false;
        if (st < T) {
          const uint32_t g = st + (uint32_t)lane;
          xj[k] = min(owner(st), 63u);
          xin[k] = g < T;
          const ExpSent sj = E.sn[xj[k]];
          xv[k] = S.ent[xin[k] ? sj.eb + g : 0];  // (every lane loads: no branch around the load)
        }
      }
      u32x3 xr[EXP_K];
#pragma unroll
      for (int k = 0; k < EXP_K; ++k) {
        const bool r = xin[k] && xv[k] >= SPLIT_EDEF && xv[k] != SPLIT_EHOLE;
        xr[k] = u32x3{0u, 0u, 0u};
        if (st0 + 64 * k < T)
          xr[k] = *reinterpret_cast<const u32x3*>(pch + (r ? (size_t)(E.sn[xj[k]].qb + (xv[k] & 0xFFFu)) : 0));
      }
#pragma unroll
      for (int k = 0; k < EXP_K; ++k) {
        const uint32_t st = st0 + 64 * k;
        if (st >= T) break;
        const uint32_t cj = xj[k], cv = xin[k] ? xv[k] : 0u;
        const bool cin = xin[k], rec = cin && cv >= SPLIT_EDEF && cv != SPLIT_EHOLE;
        // (a hole: an empty unit, no token; a direct id: one)
        const u32x3 rq = rec ? xr[k] : u32x3{cin && cv != SPLIT_EHOLE ? 1u : 0u, 0u, 0u};
        const ExpSent sj = E.sn[cj];
        const size_t ri = (size_t)(sj.qb + (cv & 0xFFFu)) * 4;
        const uint32_t cnt = rq.x;
        // tokens of the sentence before this entry: the step's exclusive sum
        // less its value at the sentence's first entry (lane e0 - st), or plus
        // the carry when the sentence began in an earlier step
        const uint32_t xex = wave_incl_add(cnt) - cnt;
        const int hl = (int)(sj.e0 - st);
        const uint32_t hb = (uint32_t)__shfl((int)xex, hl & 63);
        const uint32_t p = xex - (hl >= 0 ? hb : 0u - carry);
        // tokens this entry writes (a hole and a lane past the step: none; a
        // direct id: at most one)
        // (signed: lim and p are < 2^31)
        const int room = (int)sj.lim - (int)p;
        const uint32_t nw = room > 0 ? min(cnt, (uint32_t)room) : 0u;
        if (nw) {
          uint16_t* o = P.out_ids + sj.dst + p;
          // (the first token of a direct id and of a record in one store)
          o[0] = (uint16_t)(cv < SPLIT_EDEF ? cv : rq.y & 0xFFFFu);
          if (nw > 1) o[1] = (uint16_t)(rq.y >> 16);
          if (nw > 2) o[2] = (uint16_t)(rq.z & 0xFFFFu);
          if (nw > 3) o[3] = (uint16_t)(rq.z >> 16);
          if (nw > 4) {
            const uint16_t* pc = reinterpret_cast<const uint16_t*>(pcs + ri);
            for (uint32_t q = 4; q < nw; ++q) o[q] = pc[piece_at((int)q)];
          }
        }
        // running total of the step's last entry (its sentence may continue)
        const uint32_t ll = min(T, st + 64) - 1 - st;
        carry = lane_get(p + cnt, (int)ll);
      }
    }
    wsync();
  }
}

template <int WAVES, bool DBG, int OCC>
static hipError_t launch_scan(const TokParams& P, const SplitParams& S, int n_cu, hipStream_t s) {
  static int per_cu = 0;
  if (per_cu == 0 &&
      (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, scan_kernel<WAVES, DBG, OCC>, 64 * WAVES, 0) !=
           hipSuccess ||
       per_cu < 1))
    per_cu = 1;
  int64_t grid = (int64_t)n_cu * per_cu;
  const int64_t ng = (S.t1 - S.t0 + SUPER - 1) / SUPER;  // super-tiles
  const int64_t need = (ng + WAVES - 1) / WAVES;
  if (grid > need) grid = need;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL((scan_kernel<WAVES, DBG, OCC>), dim3((unsigned)grid), dim3(64 * WAVES), 0, s, P, S);
  return hipGetLastError();
}

template <int WAVES>
static hipError_t launch_wp(const TokParams& P, const SplitParams& S, int n_cu, hipStream_t s) {
  static int per_cu = 0;
  if (per_cu == 0 &&
      (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, wp_kernel<WAVES>, 64 * WAVES, 0) != hipSuccess ||
       per_cu < 1))
    per_cu = 1;
  const int64_t grid = (int64_t)n_cu * per_cu;
  hipLaunchKernelGGL(wp_kernel<WAVES>, dim3((unsigned)grid), dim3(64 * WAVES), 0, s, P, S);
  return hipGetLastError();
}

}  // namespace tok5

constexpr int SCAN_WAVES = 4, WP_WAVES = 12, WPT_WAVES = 8;
hipError_t finish_segment(TokParams P, const SplitParams& S, int n_cu, int fb_grid, hipStream_t s);

int64_t split_seg_slots(int64_t seg_tiles, int n_cu) {
  // 1 slot per 14 input bytes (the synthetic Wikipedia corpus queues ~0.02
  // words per byte, the CodeSearchNet-style code corpus ~0.065) + one partly
  // used chunk per scanning wave of the real grid; past it tiles fall back to
  // the serial path (counted: lddl_tokenize_stats)
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, tok5::scan_kernel<SCAN_WAVES, false, tok5::SCAN_OCC>, 64 * SCAN_WAVES,
                                                   0) != hipSuccess || per_cu < 1)
    per_cu = 8;
  const int64_t waves = (int64_t)n_cu * per_cu * SCAN_WAVES;
  const int64_t chunks = (seg_tiles * 1024 / 14 + SPLIT_CHUNK - 1) / SPLIT_CHUNK + std::min(waves, seg_tiles) + 16;
  return chunks * SPLIT_CHUNK;
}

__global__ void smeta_fallback_kernel(uint2* smeta, int64_t n_sent) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_sent; s += (int64_t)gridDim.x * blockDim.x)
    smeta[s] = make_uint2(SPLIT_NENT_FB, 0xFFFFFFFFu);
}

hipError_t launch_tokenize_serial_dense(const TokParams& P, int64_t nbytes, int64_t* tile_sent, SplitParams S,
                                        int n_cu, int fb_grid, hipStream_t s) {
  const int64_t n_tiles = tile_count(nbytes);
  hipError_t e = launch_tile_bounds(P.sent_off, P.n_sent, n_tiles, tile_sent, nullptr, s);
  if (e != hipSuccess || (e = hipMemsetAsync(P.out_tok_off, 0, sizeof(int64_t), s)) != hipSuccess) return e;
  S.tile_sent = tile_sent;
  S.t0 = 0;
  S.t1 = n_tiles;
  if ((e = launch_list_all_tiles(n_tiles, tile_sent, S.fb_list, S.fb_count, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(smeta_fallback_kernel, dim3(1024), dim3(256), 0, s, S.smeta, P.n_sent);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return finish_segment(P, S, n_cu, fb_grid, s);
}

hipError_t launch_tokenize_split(const TokParams& P, int64_t nbytes, int64_t* tile_sent, SplitParams S, int n_cu,
                                 int fb_grid, hipStream_t s, SplitTiming* tm) {
  if (tm) tm->n[0] = tm->n[1] = tm->n[2] = 0;
  auto mark = [&](int k, int side) -> hipError_t {  // (at most 64 segments timed per kernel)
    if (!tm || tm->n[k] >= 64) return hipSuccess;
    const hipError_t e = hipEventRecord(tm->ev[k][side][tm->n[k]], s);
    if (side == 1) ++tm->n[k];
    return e;
  };
  const int64_t n_tiles = tile_count(nbytes);
  const int64_t seg = S.seg_tiles > 0 ? S.seg_tiles : SPLIT_SEG_TILES;
  // (the scan reads tile_sent at its super-tile starts and the segment bounds only)
  hipError_t e = launch_tile_bounds(P.sent_off, P.n_sent, n_tiles, tile_sent, nullptr, s, seg, tok5::SUPER);
  if (e != hipSuccess) return e;
  if ((e = hipMemsetAsync(P.out_tok_off, 0, sizeof(int64_t), s)) != hipSuccess) return e;
  S.tile_sent = tile_sent;
  for (int64_t t0 = 0; t0 < n_tiles; t0 += seg) {
    S.t0 = t0;
    S.t1 = std::min(n_tiles, t0 + seg);
    if ((e = hipMemsetAsync(S.chunk_ctr, 0, 12, s)) != hipSuccess) return e;  // scan's and wp's chunk counters, scan's super-tiles
    if ((e = hipMemsetAsync(S.fb_count, 0, 4, s)) != hipSuccess) return e;
    if ((e = mark(0, 0)) != hipSuccess) return e;
    if (P.dbg) e = tok5::launch_scan<SCAN_WAVES, true, tok5::SCAN_OCC>(P, S, n_cu, s);
    else e = tok5::launch_scan<SCAN_WAVES, false, tok5::SCAN_OCC>(P, S, n_cu, s);
    if (e != hipSuccess || (e = mark(0, 1)) != hipSuccess || (e = mark(1, 0)) != hipSuccess) return e;
    // WordPiece by Bloom scan + bucket probes (default) or by trie walk
    // (LDDL_WP_ALGO=trie: A/B, slower)
    const bool trie = getenv("LDDL_WP_ALGO") && strcmp(getenv("LDDL_WP_ALGO"), "trie") == 0;
    if ((e = (trie && P.trie) ? tok5::launch_wpt<WPT_WAVES>(P, S, n_cu, s) : tok5::launch_wp<WP_WAVES>(P, S, n_cu, s)) !=
        hipSuccess)
      return e;
    if ((e = mark(1, 1)) != hipSuccess || (e = mark(2, 0)) != hipSuccess) return e;
    if ((e = finish_segment(P, S, n_cu, fb_grid, s)) != hipSuccess || (e = mark(2, 1)) != hipSuccess) return e;
  }
  return hipSuccess;
}

// The end of a segment: the serial path over the tiles the scan listed (its
// ids into the segment's entry buffer, as direct ids), the final counts, their
// exclusive scan continuing the previous segment's (out_tok_off), and the
// dense ids.
hipError_t finish_segment(TokParams P, const SplitParams& S, int n_cu, int fb_grid, hipStream_t s) {
  TokParams F = P;
  F.out_ids = S.ent - (S.t0 << 10);  // the serial path writes at sent_off[s] - sent_off[0]
  hipError_t e = launch_tokenize_fallback(F, S.fb_list, S.fb_count, fb_grid, s);
  if (e != hipSuccess) return e;
#ifndef LDDL_CNT_BLOCKS
#define LDDL_CNT_BLOCKS 256
#endif
  const int64_t cnt_grid = std::max<int64_t>(
      1, std::min<int64_t>((int64_t)n_cu * LDDL_CNT_BLOCKS, (S.seg_sent_cap + 256 * tok5::CNT_U - 1) / (256 * tok5::CNT_U)));
  hipLaunchKernelGGL(tok5::count_kernel, dim3((unsigned)cnt_grid), dim3(256), 0, s, P, S);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = launch_scan_ntok_range(P.out_ntok, S.tile_sent + S.t0, S.tile_sent + S.t1, S.seg_sent_cap, P.out_tok_off,
                                  S.scan_bsum, s)) != hipSuccess)
    return e;
  // blocks per CU of the grid-stride expand (4 waves each, far more than fit at once: the
  // hardware hands the later blocks to whichever waves finish, so each wave runs few groups and
  // the launch's tail is short): LDDL_EXP_BLOCKS (A/B), default 192 -- 16 / 32 / 96 / 192 / 768
  // measured 16.7 / 16.0 / 15.3 / 15.2 / 15.1 ms per 21.4 GB step with 8 GiB segments
  // (profiles/r6/eb/; 16 was best at 2 GiB segments in round 4); no more blocks than a block-round
  // of 256 sentences each needs
  static const int exp_blocks = [] {
    const char* v = getenv("LDDL_EXP_BLOCKS");
    const int b = v ? atoi(v) : 0;
    return b > 0 && b <= 4096 ? b : 192;
  }();
  const int64_t exp_grid = std::max<int64_t>(1, std::min<int64_t>((int64_t)n_cu * exp_blocks, (S.seg_sent_cap + 255) / 256));
  hipLaunchKernelGGL(tok5::expand_kernel, dim3((unsigned)exp_grid), dim3(256), 0, s, P, S);
  return hipGetLastError();
}

}  // namespace lddl
