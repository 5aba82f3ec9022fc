// Tokenizer v3 (default): one 256-thread workgroup per sentence-aligned tile.
//
// Same contract and results as tokenize.hip (reference: HF tokenizers'
// BertNormalizer / BertPreTokenizer / WordPiece behind
// tokenizer.tokenize(s, max_length=512, truncation=True),
// lddl/dask/bert/pretrain.py:79-80; restated in oracle/tokenizer_oracle.c).
//
// Tiles: tile t owns the sentences whose first byte lies in
// [t * TILE, (t+1) * TILE) (relative to sent_off[0]); no sentence crosses a
// tile, so every tile is independent -- no carries, no deferral, one launch
// over millions of tiles.  tile_sent[t] = first sentence of tile t
// (tile_bounds_kernel, one pass over the sentences).
//
// Per tile, all in LDS:
//   A  raw bytes -> chars: UTF-8 decode, per-code-point table (ASCII from an
//      LDS copy), literal special tokens on the raw text; every sentence start
//      (but the tile's first) inserts a boundary space into the normalised
//      stream, so words never cross sentences and a unit's sentence is the
//      count of boundary spaces before it.  Block scan -> normalised UTF-8.
//   B  units (words = runs of word chars, isolated punctuation / CJK,
//      specials) by a block-wide compaction.
//   C  WordPiece, thread per unit: greedy longest-match-first, one 16-byte
//      slot load per candidate (verified against the slot's key prefix);
//      pieces staged at the unit's normalised offset (#pieces <= #chars <=
//      #bytes, so they always fit).  (A block-synchronous variant that probes
//      all candidate lengths of a piece in parallel measured slower: git
//      history, commit "block-wide WordPiece rounds".)
//   D  segmented block scan of piece counts by sentence -> ids written
//      straight to their final slots; per-sentence counts.
// Tiles the LDS path does not model (ccc>0 survivors needing canonical
// reordering, > TRAW raw bytes, > TNB normalised bytes, > TUNITS units) are
// appended to a list and re-run by tokenize_fallback_kernel (the exact serial
// per-sentence path of tokenize.hip) right after.
#include "common.h"
#include "tokenize.h"
#include "tokenize_serial.h"

namespace lddl {

constexpr int TT = 256;         // threads per tile workgroup
constexpr int TILE_SHIFT = 10;  // nominal tile: sentences starting in 1 KiB
constexpr int TRAW = 2048;      // raw bytes of a tile kept in LDS
constexpr int TNB = 3072;       // normalised bytes (incl. boundary spaces)
constexpr int TUNITS = 1024;    // units per tile
constexpr int TSENT = 255;      // sentences per tile (u8 start counts)

enum : uint32_t { F_CLS = 3u, F_START = 4u, F_SPECIAL = 8u, F_SBND = 16u };

struct TileLds {
  uint8_t raw[TRAW + 16];
  uint8_t scount[TRAW + 16];     // #sentence starts (k >= 1) at each raw byte
  uint8_t nb[TNB + 16];
  uint8_t nf[TNB + 16];
  uint16_t piece[TNB];
  uint16_t ustart[TUNITS];
  uint16_t ucnt[TUNITS];
  uint16_t usent[TUNITS];
  uint16_t upos[TUNITS];
  uint16_t sstart[TSENT + 1];
  int32_t stot[TSENT];
  uint32_t cover[TRAW / 32 + 1]; // raw bytes consumed by a special token
  uint32_t ascii[128];
  int32_t red[2 * (TT / 64)];
  int32_t flag;
};

// exclusive block scan of two ints (256 threads)
__device__ __forceinline__ void block_scan2(TileLds& L, int a, int b, int* ea, int* eb, int* ta, int* tb) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = a, y = b;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int xa = __shfl_up(x, o), yb = __shfl_up(y, o);
    if (lane >= o) { x += xa; y += yb; }
  }
  if (lane == 63) { L.red[w] = x; L.red[4 + w] = y; }
  __syncthreads();
  int ba = 0, bb = 0, sa = 0, sb = 0;
#pragma unroll
  for (int k = 0; k < TT / 64; ++k) {
    if (k < w) { ba += L.red[k]; bb += L.red[4 + k]; }
    sa += L.red[k];
    sb += L.red[4 + k];
  }
  *ea = ba + x - a;
  *eb = bb + y - b;
  *ta = sa;
  *tb = sb;
  __syncthreads();
}

// tile_sent[t] = first sentence whose start (relative) >= t * TILE
__global__ void tile_bounds_kernel(const int64_t* sent_off, int64_t n_sent, int64_t n_tiles, int64_t* tile_sent) {
  const int64_t base = sent_off[0];
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= n_sent; s += (int64_t)gridDim.x * blockDim.x) {
    // tiles t with off[s-1] < t*TILE <= off[s] map to s (s = n_sent: the rest)
    const int64_t hi = s < n_sent ? sent_off[s] - base : (n_tiles << TILE_SHIFT);
    const int64_t lo = s > 0 ? sent_off[s - 1] - base : -1;
    int64_t t0 = (lo >> TILE_SHIFT) + 1;  // first t with t*TILE > lo
    if (lo < 0) t0 = 0;
    const int64_t t1 = hi >> TILE_SHIFT;  // last t with t*TILE <= hi
    for (int64_t t = t0; t <= t1 && t <= n_tiles; ++t) tile_sent[t] = s;
  }
}

__global__ __launch_bounds__(TT) void tokenize_tile_kernel(TokParams P, const int64_t* tile_sent, int32_t* fb_list,
                                                          int32_t* fb_count, int64_t t_base) {
  __shared__ TileLds L;
  const int tid = threadIdx.x;
  const int64_t t = t_base + blockIdx.x;
  const bool dbg = P.dbg != nullptr && tid == 0;
  uint64_t tprev = dbg ? __builtin_amdgcn_s_memtime() : 0;
#define TSTAMP(k)                                                                    \
  if (dbg) {                                                                         \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                                \
    atomicAdd((unsigned long long*)&P.dbg[k], (unsigned long long)(t_ - tprev));     \
    tprev = t_;                                                                      \
  }
  const int64_t sa = tile_sent[t], sb = tile_sent[t + 1];
  if (sa >= sb) return;
  const int64_t A = P.sent_off[sa], B = P.sent_off[sb];
  const int nraw = (int)(B - A), ns = (int)(sb - sa);
  if (nraw > TRAW || ns > TSENT) {
    if (tid == 0) fb_list[atomicAdd(fb_count, 1)] = (int32_t)t;
    return;
  }
  const int64_t base = P.sent_off[0];
  // ---- load: ascii table, sentence starts, raw bytes ----------------------
  if (tid < 128) L.ascii[tid] = P.pages[(uint32_t)P.top[0] * 256u + tid];
  for (int i = tid; i <= ns; i += TT) L.sstart[i] = (uint16_t)(P.sent_off[sa + i] - A);
  for (int i = tid; i < TRAW + 16; i += TT) {
    L.raw[i] = i < nraw ? P.bytes[A + i] : 0;
    L.scount[i] = 0;
  }
  for (int i = tid; i < TRAW / 32 + 1; i += TT) L.cover[i] = 0;
  if (tid == 0) L.flag = 0;
  __syncthreads();
  for (int i = 1 + tid; i < ns; i += TT) atomicAdd((uint32_t*)&L.scount[L.sstart[i] & ~3], 1u << (8 * (L.sstart[i] & 3)));
  TSTAMP(0);
  // ---- A1: char starts, entries, specials ---------------------------------
  constexpr int RPT = TRAW / TT;  // raw bytes per thread (8)
  uint32_t ent[RPT], cpv[RPT];
  bool ok[RPT];
  bool hard = false;
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int i = tid * RPT + k;
    const uint32_t b = L.raw[i];
    ok[k] = false;
    ent[k] = 0;
    cpv[k] = b;
    if (i >= nraw || (b & 0xC0u) == 0x80u) continue;
    ok[k] = true;
    if (b < 0x80) {
      ent[k] = L.ascii[b];
      if (b == '[') {
        // special literal inside its sentence: sentence end = next start > i
        int lo = 0, hi = ns;  // first sentence index with sstart > i
        while (lo < hi) { const int m = (lo + hi) >> 1; if (L.sstart[m] <= i) lo = m + 1; else hi = m; }
        const int lim = lo < ns ? L.sstart[lo] : nraw;
        int len = 0, sk = -1;
        if (i + 5 <= lim) {
          const uint32_t c1 = L.raw[i + 1], c2 = L.raw[i + 2], c3 = L.raw[i + 3], c4 = L.raw[i + 4];
          if (c1 == 'P' && c2 == 'A' && c3 == 'D' && c4 == ']') { sk = 0; len = 5; }
          else if (c1 == 'U' && c2 == 'N' && c3 == 'K' && c4 == ']') { sk = 1; len = 5; }
          else if (c1 == 'C' && c2 == 'L' && c3 == 'S' && c4 == ']') { sk = 2; len = 5; }
          else if (c1 == 'S' && c2 == 'E' && c3 == 'P' && c4 == ']') { sk = 3; len = 5; }
          else if (c1 == 'M' && c2 == 'A' && c3 == 'S' && c4 == 'K' && i + 6 <= lim && L.raw[i + 5] == ']') { sk = 4; len = 6; }
        }
        if (sk >= 0) {
          ent[k] = 0xF0000000u | ((uint32_t)sk << 8) | (uint32_t)len;
          for (int q = 1; q < len; ++q) atomicOr(&L.cover[(i + q) >> 5], 1u << ((i + q) & 31));
        }
      }
    } else {
      const int a = utf8_len(b);
      uint32_t cp = b & (0x3Fu >> (a - 1));
      for (int q = 1; q < a; ++q) cp = (cp << 6) | (L.raw[i + q] & 0x3Fu);
      if (cp > 0x10FFFF) cp = 0xFFFD;
      cpv[k] = cp;
      ent[k] = table_entry(P, cp);
      bool h = ent_rank(ent[k]) != 0;
      if (ent_kind(ent[k]) == KIND_MULTI) {
        const uint4 m = P.multi[ent_payload(ent[k])];
        h = h || (ent_rank(m.y) | ent_rank(m.z) | ent_rank(m.w)) != 0;
      }
      hard = hard || h;
    }
  }
  if (hard) L.flag = 1;
  __syncthreads();
  if (L.flag) {
    if (tid == 0) fb_list[atomicAdd(fb_count, 1)] = (int32_t)t;
    return;
  }
  TSTAMP(1);
  // ---- A2: output sizes (+ boundary spaces), block scan, write ------------
  int nout[RPT], my = 0;
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int i = tid * RPT + k;
    nout[k] = 0;
    if (i < nraw) my += L.scount[i];  // boundary spaces before this byte
    if (!ok[k]) continue;
    const bool isspec = (ent[k] >> 28) == 0xFu;
    if (!isspec && ((L.cover[i >> 5] >> (i & 31)) & 1u)) { ok[k] = false; continue; }
    if (isspec) { nout[k] = 1; my += 1; continue; }
    const uint32_t kind = ent_kind(ent[k]);
    if (kind == KIND_DROP_T || kind == KIND_DROP_D) continue;
    if (kind == KIND_MULTI) {
      const uint4 m = P.multi[ent_payload(ent[k])];
      nout[k] = utf8_enc_len(ent_payload(m.y)) + utf8_enc_len(ent_payload(m.z)) +
                (m.x > 2 ? utf8_enc_len(ent_payload(m.w)) : 0);
    } else {
      nout[k] = utf8_enc_len(kind == KIND_IDENT ? cpv[k] : ent_payload(ent[k]));
    }
    my += nout[k];
  }
  int obeg, dummy, nlen, dummy2;
  block_scan2(L, my, 0, &obeg, &dummy, &nlen, &dummy2);
  if (nlen > TNB) {
    if (tid == 0) fb_list[atomicAdd(fb_count, 1)] = (int32_t)t;
    return;
  }
  {
    int o = obeg;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int i = tid * RPT + k;
      if (i < nraw)
        for (int q = L.scount[i]; q > 0; --q) { L.nb[o] = ' '; L.nf[o] = F_SBND | F_START | CLS_SPACE; ++o; }
      if (!ok[k] || (nout[k] == 0)) continue;
      if ((ent[k] >> 28) == 0xFu) {
        L.nb[o] = (uint8_t)((ent[k] >> 8) & 0xF);
        L.nf[o] = F_SPECIAL | F_START | CLS_ISOLATE;
        ++o;
        continue;
      }
      const uint32_t kind = ent_kind(ent[k]);
      uint32_t ch[3] = {0, 0, 0};
      int nc = 1;
      uint32_t cls = ent_cls(ent[k]);
      if (kind == KIND_MULTI) {
        const uint4 m = P.multi[ent_payload(ent[k])];
        ch[0] = ent_payload(m.y); ch[1] = ent_payload(m.z); ch[2] = ent_payload(m.w);
        nc = (int)m.x;
        cls = CLS_OTHER;
      } else {
        ch[0] = kind == KIND_IDENT ? cpv[k] : ent_payload(ent[k]);
      }
      for (int q = 0; q < nc; ++q) {
        const uint32_t c = ch[q];
        const int l = utf8_enc_len(c);
        uint32_t u8;
        if (l == 1) u8 = c;
        else if (l == 2) u8 = (0xC0 | (c >> 6)) | ((0x80 | (c & 0x3F)) << 8);
        else if (l == 3) u8 = (0xE0 | (c >> 12)) | ((0x80 | ((c >> 6) & 0x3F)) << 8) | ((0x80 | (c & 0x3F)) << 16);
        else u8 = (0xF0 | (c >> 18)) | ((0x80 | ((c >> 12) & 0x3F)) << 8) | ((0x80 | ((c >> 6) & 0x3F)) << 16) |
                  ((0x80 | (c & 0x3F)) << 24);
        for (int q2 = 0; q2 < l; ++q2) {
          L.nb[o] = (uint8_t)(u8 >> (8 * q2));
          L.nf[o] = (uint8_t)(cls | (q2 == 0 ? F_START : 0u));
          ++o;
        }
      }
    }
  }
  __syncthreads();
  TSTAMP(2);
  // ---- B: units + sentence of each unit (block compaction) ---------------
  constexpr int NPT = TNB / TT;  // normalised bytes per thread (12)
  uint32_t um = 0;
  int sb_local = 0;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int j = tid * NPT + k;
    if (j >= nlen) break;
    const uint32_t f = L.nf[j];
    if (f & F_SBND) { ++sb_local; continue; }
    if (!(f & F_START)) continue;
    const uint32_t c = f & F_CLS;
    bool st = (f & F_SPECIAL) || c == CLS_ISOLATE;
    if (c == CLS_OTHER && !(f & F_SPECIAL))
      st = j == 0 || (L.nf[j - 1] & (F_CLS | F_SPECIAL)) != CLS_OTHER;
    if (st) um |= 1u << k;
  }
  int ubeg, sbeg, nunits, nsb;
  block_scan2(L, __popc(um), sb_local, &ubeg, &sbeg, &nunits, &nsb);
  if (nunits > TUNITS) {
    if (tid == 0) fb_list[atomicAdd(fb_count, 1)] = (int32_t)t;
    return;
  }
  {
    int u = ubeg, sc = sbeg;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int j = tid * NPT + k;
      if (j >= nlen) break;
      if (L.nf[j] & F_SBND) { ++sc; continue; }
      if (um & (1u << k)) { L.ustart[u] = (uint16_t)j; L.usent[u] = (uint16_t)sc; ++u; }
    }
  }
  for (int i = tid; i < ns; i += TT) L.stot[i] = 0;
  __syncthreads();
  TSTAMP(3);
  // ---- C: WordPiece, thread per unit --------------------------------------
  for (int u = tid; u < nunits; u += TT) {
    const int j = L.ustart[u];
    const uint32_t f = L.nf[j];
    int cnt;
    if (f & F_SPECIAL) {
      L.piece[j] = (uint16_t)P.special[L.nb[j]];
      cnt = 1;
    } else {
      int e = j + 1, nch = 1;
      if ((f & F_CLS) == CLS_OTHER) {
        while (e < nlen && (L.nf[e] & (F_CLS | F_SPECIAL)) == CLS_OTHER) {
          nch += (L.nf[e] & F_START) ? 1 : 0;
          ++e;
        }
      } else {
        while (e < nlen && !(L.nf[e] & F_START)) ++e;
      }
      cnt = -1;
      if (nch <= 100) {
        auto get = [&](int i) -> uint32_t { return L.nb[j + i]; };
        auto em = [&](int n, uint32_t id) { L.piece[j + n] = (uint16_t)id; };
        cnt = wordpiece_core(P, get, e - j, em);
      }
      if (cnt < 0) {
        L.piece[j] = (uint16_t)P.unk;
        cnt = 1;
      }
    }
    L.ucnt[u] = (uint16_t)cnt;
  }
  __syncthreads();
  TSTAMP(4);
  TSTAMP(7);
  // ---- D: token index inside the sentence (segmented scan) ---------------
  constexpr int UPT = TUNITS / TT;  // units per thread (4), contiguous
  int run = 0, headseen = 0;
  int lsum[UPT];
  const int u0 = tid * UPT;
#pragma unroll
  for (int k = 0; k < UPT; ++k) {
    const int u = u0 + k;
    lsum[k] = 0;
    if (u >= nunits) continue;
    if (u == 0 || L.usent[u] != L.usent[u - 1]) { run = 0; headseen = 1; }
    lsum[k] = run;  // exclusive within the thread's segment piece
    run += L.ucnt[u];
  }
  // carry from previous threads: sum of counts since the last segment head
  // before u0 -- block scan of (headseen, run) with segmented combine
  {
    const int lane = tid & 63, w = tid >> 6;
    int hv = headseen, sv = run;  // this thread's (has head, tail sum)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int ph = __shfl_up(hv, o), ps = __shfl_up(sv, o);
      if (lane >= o && !hv) { sv += ps; hv = ph; }
    }
    // per-wave inclusive (hv, sv); combine across waves
    if (lane == 63) { L.red[w] = sv; L.red[4 + w] = hv; }
    __syncthreads();
    int carry_s = 0, carry_h = 0;
    for (int k = w - 1; k >= 0 && !carry_h; --k) {
      carry_s += L.red[k];
      carry_h = L.red[4 + k];
    }
    // exclusive value for this thread = inclusive of previous thread
    int ex_s = __shfl_up(sv, 1), ex_h = __shfl_up(hv, 1);
    if (lane == 0) { ex_s = 0; ex_h = 0; }
    if (!ex_h) ex_s += carry_s;
    // units of this thread before its first head continue the carried sum
    bool before_head = true;
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int u = u0 + k;
      if (u >= nunits) continue;
      if (u == 0 || L.usent[u] != L.usent[u - 1]) before_head = false;
      L.upos[u] = (uint16_t)min(lsum[k] + (before_head ? ex_s : 0), 65535);
    }
    __syncthreads();
  }
  TSTAMP(8);
  // ---- write ids and per-sentence counts ----------------------------------
  for (int u = tid; u < nunits; u += TT) {
    const int s = L.usent[u];
    const int c = L.ucnt[u];
    const int t0 = L.upos[u];
    const int64_t ob = A + L.sstart[s] - base;
    const int j = L.ustart[u];
    for (int q = 0; q < c; ++q)
      if (t0 + q < P.max_tok) P.out_ids[ob + t0 + q] = L.piece[j + q];
    if (u == nunits - 1 || L.usent[u + 1] != s) L.stot[s] = t0 + c;
  }
  __syncthreads();
  for (int i = tid; i < ns; i += TT) P.out_ntok[sa + i] = min(L.stot[i], P.max_tok);
  TSTAMP(9);
  if (dbg) atomicAdd((unsigned long long*)&P.dbg[11], 1ull);
#undef TSTAMP
}

// Exact serial path for the listed tiles: lane per sentence (tokenize.hip).
__global__ __launch_bounds__(256) void tokenize_fallback_kernel(TokParams P, const int64_t* tile_sent,
                                                                const int32_t* fb_list, const int32_t* fb_count) {
  __shared__ uint32_t ascii_tab[128];
  if (threadIdx.x < 128) ascii_tab[threadIdx.x] = P.pages[(uint32_t)P.top[0] * 256u + threadIdx.x];
  __syncthreads();
  const int n = *fb_count;
  const LdsWordBuf wb{P.ovf + ((size_t)blockIdx.x * 256 + threadIdx.x) * WB_OVF};
  const int64_t base = P.sent_off[0];
  const int wave = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const int nw = (gridDim.x * 256) >> 6;
  for (int k = wave; k < n; k += nw) {
    const int64_t t = fb_list[k];
    const int64_t sa = tile_sent[t], sb = tile_sent[t + 1];
    for (int64_t s = sa + lane; s < sb; s += 64) {
      SentState st{P.sent_off[s], P.sent_off[s + 1], P.sent_off[s] - base, 0};
      while (st.p < st.e && st.ntok < P.max_tok) step(P, st, wb, ascii_tab);
      P.out_ntok[s] = min(st.ntok, P.max_tok);
    }
  }
}

int64_t tile_count(int64_t nbytes) { return (nbytes >> TILE_SHIFT) + 1; }

// The dispatch packet's grid size is 32-bit in work-items, so a launch of
// more than 2^32 / TT tiles would wrap: tiles go out in chunks of at most
// `chunk` workgroups (default 2^22, i.e. 4 GiB of input per launch).
hipError_t launch_tokenize_tiles(const TokParams& P, int64_t nbytes, int64_t* tile_sent, int32_t* fb_list,
                                 int32_t* fb_count, int fb_grid, int64_t chunk, hipStream_t s) {
  const int64_t n_tiles = tile_count(nbytes);
  hipError_t e = launch_tile_bounds(P.sent_off, P.n_sent, n_tiles, tile_sent, s);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(fb_count, 0, 4, s);
  if (e != hipSuccess) return e;
  if (chunk <= 0 || chunk > (int64_t(1) << 22)) chunk = int64_t(1) << 22;
  for (int64_t t0 = 0; t0 < n_tiles; t0 += chunk) {
    const int64_t nt = n_tiles - t0 < chunk ? n_tiles - t0 : chunk;
    hipLaunchKernelGGL(tokenize_tile_kernel, dim3((unsigned)nt), dim3(TT), 0, s, P, tile_sent, fb_list, fb_count, t0);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return launch_tokenize_fallback(P, tile_sent, fb_list, fb_count, fb_grid, s);
}

hipError_t launch_tile_bounds(const int64_t* sent_off, int64_t n_sent, int64_t n_tiles, int64_t* tile_sent,
                              hipStream_t s) {
  hipLaunchKernelGGL(tile_bounds_kernel, dim3(4096), dim3(256), 0, s, sent_off, n_sent, n_tiles, tile_sent);
  return hipGetLastError();
}

hipError_t launch_tokenize_fallback(const TokParams& P, const int64_t* tile_sent, const int32_t* fb_list,
                                    const int32_t* fb_count, int grid, hipStream_t s) {
  hipLaunchKernelGGL(tokenize_fallback_kernel, dim3(grid), dim3(256), 0, s, P, tile_sent, fb_list, fb_count);
  return hipGetLastError();
}

}  // namespace lddl
