// WordPiece tokenizer for gfx950: BertNormalizer + BertPreTokenizer +
// WordPiece(greedy longest-match-first) + per-sentence truncation.
//
// Replaces the per-sentence call tokenizer.tokenize(s, max_length=512,
// truncation=True) of lddl/dask/bert/pretrain.py:79-80 (and
// pretrain_codebert.py:123-124), i.e. HF tokenizers' BertNormalizer /
// BertPreTokenizer / WordPiece as configured by BertTokenizerFast(vocab_file)
// (pretrain.py:584-587).  Algorithm restated in oracle/tokenizer_oracle.c.
//
// Layout in HBM
//   bytes     u8 [nbytes + 16 pad]      sentences back to back (UTF-8)
//   sent_off  i64[n_sent + 1]
//   out_ids   u16[nbytes]  sentence s writes its ids at sent_off[s]-sent_off[0]
//                          (#tokens <= #bytes for every input, so no scan)
//   out_ntok  i32[n_sent]  min(#tokens, max_tok)
//
// Two kernels, both exact:
//  * tokenize_wave_kernel (default): a wave owns a chunk of consecutive
//    sentences and walks it in raw windows of WIN bytes.  Per window the 64
//    lanes load the bytes coalesced, decode UTF-8 and look every char up in
//    the per-code-point table in parallel, write the normalised UTF-8 into LDS
//    (wave prefix scan), find word / punctuation / special units (ballot
//    compaction), run WordPiece lane-per-unit against the vocab hash, and
//    scatter the ids with a second scan.  A word cut by the window end is
//    deferred to the next window.  Inputs the window path does not model
//    (canonical reordering of ccc>0 survivors, a word longer than a window,
//    more than PSTAGE pieces on one lane) fall back to the serial path for
//    that one sentence, on lane 0 of the same wave.
//  * tokenize_kernel: one lane per sentence, word by word (the serial path;
//    kept for A/B).  Lanes of a wave pull sentences dynamically (ballot
//    refill) so lognormal sentence lengths do not idle the wave.
// WordPiece in both: O(1)-shrinking polynomial hash probed in an L2-resident
// table, every hit verified byte-exactly against the vocab pool.
#include "common.h"
#include "tokenize.h"
#include "tokenize_serial.h"

namespace lddl {

__global__ __launch_bounds__(BLOCK) void tokenize_kernel(TokParams P) {
  __shared__ uint32_t ascii_tab[128];
  if (threadIdx.x < 128) ascii_tab[threadIdx.x] = P.pages[(uint32_t)P.top[0] * 256u + threadIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const LdsWordBuf wb{P.ovf + ((size_t)blockIdx.x * BLOCK + threadIdx.x) * WB_OVF};
  const int64_t base = P.sent_off[0];
  for (;;) {
    uint32_t chunk = 0;
    if (lane == 0) chunk = atomicAdd(P.work_counter, 1u);
    chunk = __shfl(chunk, 0);
    const int64_t lo = (int64_t)chunk * P.chunk;
    if (lo >= P.n_sent) break;
    const int64_t hi = min(lo + (int64_t)P.chunk, P.n_sent);
    int64_t next = lo + 64;
    int64_t s = lo + lane;
    bool active = s < hi;
    SentState st{};
    if (active) { st.p = P.sent_off[s]; st.e = P.sent_off[s + 1]; st.obase = st.p - base; st.ntok = 0; }
    while (__ballot(active)) {
      bool fin = false;
      if (active) {
        step(P, st, wb, ascii_tab);
        fin = st.p >= st.e || st.ntok >= P.max_tok;
        if (fin) P.out_ntok[s] = min(st.ntok, P.max_tok);
      }
      const uint64_t m = __ballot(fin);
      if (m) {
        const int r = __popcll(m & ((1ull << lane) - 1ull));
        if (fin) {
          s = next + r;
          active = s < hi;
          if (active) { st.p = P.sent_off[s]; st.e = P.sent_off[s + 1]; st.obase = st.p - base; st.ntok = 0; }
        }
        next += __popcll(m);
      }
    }
  }
}

// --------------------------------------------------------------------------
// v2: wave-cooperative windows (default).  A wave (= one workgroup) owns a
// chunk of consecutive sentences and walks it in raw windows of WIN bytes.
// --------------------------------------------------------------------------
constexpr int WIN = 256;             // raw bytes per window (one dword per lane)
constexpr int NBCAP = 3 * WIN + 16;  // normalised bytes (<= 3x expansion)
constexpr int PSTAGE = 24;           // staged pieces per lane per window
constexpr int64_t I64MAX = 0x7fffffffffffffffLL;

// flags of a normalised byte (every byte of a char carries the char's flags)
enum : uint32_t { NF_CLS = 3u, NF_START = 4u, NF_SPECIAL = 8u };

struct WaveLds {
  uint8_t raw[WIN + 16];        // raw bytes [base4, base4 + WIN + 16)
  uint8_t nb[NBCAP];            // normalised UTF-8 (special: its index 0..4)
  uint8_t nf[NBCAP];            // flags
  uint8_t nord[NBCAP];          // sentence ordinal of the char
  uint16_t nraw[NBCAP];         // raw offset (from base4) of the owning char
  uint16_t ustart[WIN];         // unit start (normalised offset); a unit
  uint16_t ucnt[WIN];           //   covers >= 1 raw byte, so <= WIN units
  uint16_t ustage[WIN];         // unit's first staged piece (lane-local)
  uint16_t upos[WIN];           // unit's first token index in the window
  uint16_t stage[64][PSTAGE];   // staged piece ids per lane
  int64_t sst[64];              // starts of sentences sc+1 .. sc+64
  int32_t ordcnt[65];           // tokens per sentence ordinal in the window
  int32_t ordfirst[65];         // window token index of an ordinal's first unit
};

__device__ __forceinline__ int wave_excl_scan(int v, int lane, int* total) {
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  *total = __shfl(x, 63);
  return x - v;
}

__device__ __forceinline__ int64_t wave_min64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t y = __shfl_xor(v, o);
    v = y < v ? y : v;
  }
  return v;
}

// number of sentence starts <= pos among sst[0..63] (sorted ascending)
__device__ __forceinline__ int ordinal_of(const WaveLds& L, int64_t pos) {
  int lo = 0, hi = 64;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (L.sst[mid] <= pos) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// literal special token at raw window index i (raw[i] == '['), ending <= lim
__device__ __forceinline__ int match_special_lds(const WaveLds& L, int i, int lim, int* len) {
  if (i + 5 > lim) return -1;
  const uint32_t c1 = L.raw[i + 1], c2 = L.raw[i + 2], c3 = L.raw[i + 3], c4 = L.raw[i + 4];
  if (c1 == 'P' && c2 == 'A' && c3 == 'D' && c4 == ']') { *len = 5; return 0; }
  if (c1 == 'U' && c2 == 'N' && c3 == 'K' && c4 == ']') { *len = 5; return 1; }
  if (c1 == 'C' && c2 == 'L' && c3 == 'S' && c4 == ']') { *len = 5; return 2; }
  if (c1 == 'S' && c2 == 'E' && c3 == 'P' && c4 == ']') { *len = 5; return 3; }
  if (c1 == 'M' && c2 == 'A' && c3 == 'S' && c4 == 'K' && i + 6 <= lim && L.raw[i + 5] == ']') { *len = 6; return 4; }
  return -1;
}

__device__ __forceinline__ void load_sst(WaveLds& L, const TokParams& P, int64_t sc, int64_t s_hi, int lane) {
  const int64_t j = sc + 1 + lane;
  L.sst[lane] = j <= s_hi ? P.sent_off[j] : I64MAX;
}

// LDS ordering between lanes of ONE wave (waves of a workgroup run
// independent chunks, so no workgroup barrier inside the loop)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(64 * TOK_WAVES) void tokenize_wave_kernel(TokParams P) {
  __shared__ WaveLds Ls[TOK_WAVES];
  __shared__ uint32_t ascii_tab[128];
  __shared__ uint32_t bloom[BLOOM_WORDS];  // exact-negative filter of vocab keys
  for (int i = threadIdx.x; i < BLOOM_WORDS; i += 64 * TOK_WAVES) bloom[i] = P.bloom[i];
  if (threadIdx.x < 128) ascii_tab[threadIdx.x] = P.pages[(uint32_t)P.top[0] * 256u + threadIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  WaveLds& L = Ls[wave];
  auto filt = [&](uint64_t key) -> bool {
    const uint32_t w = bloom[(uint32_t)(key >> 40) & (BLOOM_WORDS - 1)];
    return ((w >> (key & 31)) & (w >> ((key >> 5) & 31)) & 1u) != 0;
  };
  const int64_t base = P.sent_off[0];
  const int64_t data_end = P.sent_off[P.n_sent];
  const GlobalWordBuf fb{P.ovf + ((size_t)blockIdx.x * TOK_WAVES + wave) * (WB_LDS + WB_OVF)};
  const bool dbg = P.dbg != nullptr;
  uint64_t acc[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tprev = dbg ? __builtin_amdgcn_s_memtime() : 0;
#define STAMP(k)                                        \
  if (dbg) {                                            \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();   \
    acc[k] += t_ - tprev;                               \
    tprev = t_;                                         \
  }
  for (;;) {
    uint32_t chunk = 0;
    if (lane == 0) chunk = atomicAdd(P.work_counter, 1u);
    chunk = __shfl(chunk, 0);
    const int64_t s_lo = (int64_t)chunk * P.chunk;
    if (s_lo >= P.n_sent) break;
    const int64_t s_hi = min(s_lo + (int64_t)P.chunk, P.n_sent);
    const int64_t chunk_end = P.sent_off[s_hi];
    int64_t sc = s_lo;               // current sentence
    int64_t cur = P.sent_off[s_lo];  // next unprocessed raw byte
    int32_t stok = 0;                // tokens of sentence sc emitted so far
    load_sst(L, P, sc, s_hi, lane);
    wave_sync();
    while (sc < s_hi) {
      const int64_t base4 = cur & ~(int64_t)3;
      const int64_t wend = min(base4 + WIN, chunk_end);
      STAMP(0);
      if (dbg) acc[8] += 1;
      // ---- raw bytes [base4, base4 + WIN + 16), bounded by the data -------
      {
        const int64_t a = base4 + 4 * lane;
        uint32_t v = 0;
        if (a + 4 <= data_end) v = *reinterpret_cast<const uint32_t*>(P.bytes + a);
        else for (int q = 0; q < 4; ++q) if (a + q < data_end) v |= (uint32_t)P.bytes[a + q] << (8 * q);
        *reinterpret_cast<uint32_t*>(&L.raw[4 * lane]) = v;
        if (lane < 4) {
          const int64_t a2 = base4 + WIN + 4 * lane;
          uint32_t w = 0;
          for (int q = 0; q < 4; ++q) if (a2 + q < data_end) w |= (uint32_t)P.bytes[a2 + q] << (8 * q);
          *reinterpret_cast<uint32_t*>(&L.raw[WIN + 4 * lane]) = w;
        }
      }
      wave_sync();
      STAMP(1);
      // ---- pass A: char starts, table entries, effective window end -------
      uint32_t ent[4], cps[4];
      bool ok[4], spec[4];
      int64_t cut = wend, hard_pos = I64MAX;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = 4 * lane + k;
        const int64_t pos = base4 + i;
        const uint32_t b = L.raw[i];
        ok[k] = false;
        spec[k] = false;
        ent[k] = 0;
        cps[k] = b;
        if (pos < cur || pos >= wend || (b & 0xC0u) == 0x80u) continue;
        const int a = utf8_len(b);
        if (wend < chunk_end && (pos + a > wend || (b == '[' && pos + 6 > wend))) { cut = min(cut, pos); continue; }
        ok[k] = true;
        if (b < 0x80) {
          ent[k] = ascii_tab[b];
        } else {
          uint32_t cp = b & (0x3Fu >> (a - 1));
          for (int q = 1; q < a; ++q) cp = (cp << 6) | (L.raw[i + q] & 0x3Fu);
          if (cp > 0x10FFFF) cp = 0xFFFD;
          cps[k] = cp;
          ent[k] = table_entry(P, cp);
          bool h = ent_rank(ent[k]) != 0;
          if (ent_kind(ent[k]) == KIND_MULTI) {
            const uint4 m = P.multi[ent_payload(ent[k])];
            h = h || (ent_rank(m.y) | ent_rank(m.z) | ent_rank(m.w)) != 0;
          }
          if (h) hard_pos = min(hard_pos, pos);
        }
      }
      int64_t wend_eff = wave_min64(min(cut, L.sst[63]));
      // a ccc>0 survivor (canonical reordering): stop before its sentence,
      // or run the serial fallback when it is in the current sentence
      bool fallback = false;
      const int64_t hp = wave_min64(hard_pos);
      if (hp < wend_eff) {
        const int o = ordinal_of(L, hp);
        if (o == 0) fallback = true;
        else wend_eff = min(wend_eff, L.sst[o - 1]);
      }
      int64_t cur_new = max(wend_eff, cur);
      int ntot = 0, nunits = 0;
      if (!fallback) {
        STAMP(2);
        // ---- pass B: specials (raw text, inside their sentence) ----------
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int i = 4 * lane + k;
          const int64_t pos = base4 + i;
          if (!ok[k] || pos >= wend_eff) { ok[k] = false; continue; }
          if (cps[k] == '[') {
            const int o = ordinal_of(L, pos);
            const int64_t send = min(o < 64 ? L.sst[o] : I64MAX, chunk_end);
            int sl;
            const int sk = match_special_lds(L, i, (int)min(send - base4, (int64_t)(WIN + 16)), &sl);
            if (sk >= 0) { spec[k] = true; ent[k] = ((uint32_t)sk << 8) | (uint32_t)sl; }
          }
        }
        wave_sync();
        // bytes covered by a special emit nothing: clear them in raw[] (the
        // covered chars are ASCII, in this lane or the next)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (spec[k])
            for (int q = 1; q < (int)(ent[k] & 0xFF); ++q) L.raw[4 * lane + k + q] = 0;
        wave_sync();
        int nout[4], my = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          nout[k] = 0;
          if (!ok[k]) continue;
          if (spec[k]) { nout[k] = 1; my += 1; continue; }
          if (L.raw[4 * lane + k] == 0 && cps[k] != 0) { ok[k] = false; continue; }  // inside a special
          const uint32_t kind = ent_kind(ent[k]);
          if (kind == KIND_DROP_T || kind == KIND_DROP_D) continue;
          if (kind == KIND_MULTI) {
            const uint4 m = P.multi[ent_payload(ent[k])];
            nout[k] = utf8_enc_len(ent_payload(m.y)) + utf8_enc_len(ent_payload(m.z)) +
                      (m.x > 2 ? utf8_enc_len(ent_payload(m.w)) : 0);
          } else {
            nout[k] = utf8_enc_len(kind == KIND_IDENT ? cps[k] : ent_payload(ent[k]));
          }
          my += nout[k];
        }
        const int obeg = wave_excl_scan(my, lane, &ntot);
        // ---- write normalised bytes + flags --------------------------------
        int o = obeg;
        int ord = -1;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (!ok[k] || nout[k] == 0) continue;
          const int i = 4 * lane + k;
          const int64_t pos = base4 + i;
          if (ord < 0) ord = ordinal_of(L, pos);
          while (ord < 64 && L.sst[ord] <= pos) ++ord;
          if (spec[k]) {
            L.nb[o] = (uint8_t)(ent[k] >> 8);
            L.nf[o] = NF_SPECIAL | NF_START | CLS_ISOLATE;
            L.nord[o] = (uint8_t)ord;
            L.nraw[o] = (uint16_t)i;
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
            ch[0] = kind == KIND_IDENT ? cps[k] : ent_payload(ent[k]);
          }
          for (int q = 0; q < nc; ++q) {
            const uint32_t c = ch[q];
            const int l = utf8_enc_len(c);
            uint32_t u8;
            if (l == 1) u8 = c;
            else if (l == 2) u8 = (0xC0 | (c >> 6)) | ((0x80 | (c & 0x3F)) << 8);
            else if (l == 3) u8 = (0xE0 | (c >> 12)) | ((0x80 | ((c >> 6) & 0x3F)) << 8) | ((0x80 | (c & 0x3F)) << 16);
            else u8 = (0xF0 | (c >> 18)) | ((0x80 | ((c >> 12) & 0x3F)) << 8) |
                      ((0x80 | ((c >> 6) & 0x3F)) << 16) | ((0x80 | (c & 0x3F)) << 24);
            for (int q2 = 0; q2 < l; ++q2) {
              L.nb[o] = (uint8_t)(u8 >> (8 * q2));
              L.nf[o] = (uint8_t)(cls | (q2 == 0 ? NF_START : 0u));
              L.nord[o] = (uint8_t)ord;
              L.nraw[o] = (uint16_t)i;
              ++o;
            }
          }
        }
        wave_sync();
        STAMP(3);
        // ---- units: words (runs of OTHER chars inside one sentence),
        //      isolated chars and specials, compacted in order --------------
        for (int r0 = 0; r0 < ntot; r0 += 256) {
          uint32_t sm = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int j = r0 + 4 * lane + k;
            if (j >= ntot) break;
            const uint32_t f = L.nf[j];
            if (!(f & NF_START)) continue;
            const uint32_t c = f & NF_CLS;
            bool st = (f & NF_SPECIAL) || c == CLS_ISOLATE;
            if (c == CLS_OTHER) {
              st = j == 0 || (L.nf[j - 1] & (NF_CLS | NF_SPECIAL)) != CLS_OTHER || L.nord[j - 1] != L.nord[j];
            }
            if (st) sm |= 1u << k;
          }
          int tot;
          int at = nunits + wave_excl_scan(__popc(sm), lane, &tot);
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (sm & (1u << k)) L.ustart[at++] = (uint16_t)(r0 + 4 * lane + k);
          nunits += tot;
        }
        wave_sync();
        // ---- a word cut by the window end is deferred to the next window --
        if (nunits > 0 && wend_eff < chunk_end) {
          const int j = L.ustart[nunits - 1];
          if ((L.nf[j] & (NF_CLS | NF_SPECIAL)) == CLS_OTHER) {
            int e = j + 1;
            while (e < ntot && (L.nf[e] & (NF_CLS | NF_SPECIAL)) == CLS_OTHER && L.nord[e] == L.nord[j]) ++e;
            if (e == ntot) {
              const int o2 = L.nord[j];
              bool complete = wend_eff >= (o2 < 64 ? L.sst[o2] : I64MAX);
              if (!complete) {
                const uint32_t b0 = L.raw[wend_eff - base4];  // next raw char
                if (b0 < 0x80 && b0 != 0) {
                  const uint32_t c = ent_cls(ascii_tab[b0]);
                  complete = ent_kind(ascii_tab[b0]) != KIND_DROP_T && (c == CLS_SPACE || c == CLS_ISOLATE);
                }
              }
              if (!complete) {
                cur_new = base4 + L.nraw[j];
                --nunits;
                if (cur_new <= cur) fallback = true;  // a word longer than the window
              }
            }
          }
        }
      }
      if (!fallback) {
        STAMP(4);
        if (dbg) acc[9] += nunits;
        // ---- WordPiece, lane per unit -------------------------------------
        L.ordcnt[lane] = 0;
        if (lane == 0) L.ordcnt[64] = 0;
        wave_sync();
        int used = 0;
        bool ovfl = false;
        for (int u = lane; u < nunits; u += 64) {
          const int j = L.ustart[u];
          const uint32_t f = L.nf[j];
          int cnt;
          L.ustage[u] = (uint16_t)used;
          if (f & NF_SPECIAL) {
            if (used < PSTAGE) L.stage[lane][used] = (uint16_t)P.special[L.nb[j]];
            cnt = 1;
          } else {
            int e = j + 1, nch = 1;
            if ((f & NF_CLS) == CLS_OTHER) {
              while (e < ntot && (L.nf[e] & (NF_CLS | NF_SPECIAL)) == CLS_OTHER && L.nord[e] == L.nord[j]) {
                nch += (L.nf[e] & NF_START) ? 1 : 0;
                ++e;
              }
            } else {
              while (e < ntot && !(L.nf[e] & NF_START)) ++e;
            }
            cnt = -1;
            if (P.dbg_mode == 1) {
              if (used < PSTAGE) L.stage[lane][used] = (uint16_t)P.unk;
              cnt = 1;
            } else if (nch <= 100) {
              auto get = [&](int i) -> uint32_t { return L.nb[j + i]; };
              auto em = [&](int n, uint32_t id) { if (used + n < PSTAGE) L.stage[lane][used + n] = (uint16_t)id; };
              cnt = wordpiece_core(P, get, e - j, em, filt);
            }
            if (cnt < 0) {
              if (used < PSTAGE) L.stage[lane][used] = (uint16_t)P.unk;
              cnt = 1;
            }
          }
          if (used + cnt > PSTAGE) ovfl = true;
          used += cnt;
          L.ucnt[u] = (uint16_t)cnt;
          atomicAdd(&L.ordcnt[L.nord[j]], cnt);
        }
        fallback = __ballot(ovfl) != 0;
        wave_sync();
        if (!fallback) {
          STAMP(5);
          // ---- window token index of every unit (scan over units) ---------
          int carry = 0;
          for (int r0 = 0; r0 < nunits; r0 += 64) {
            const int u = r0 + lane;
            const int c = u < nunits ? L.ucnt[u] : 0;
            int tot;
            const int pre = carry + wave_excl_scan(c, lane, &tot);
            if (u < nunits) {
              const int o = L.nord[L.ustart[u]];
              if (u == 0 || L.nord[L.ustart[u - 1]] != o) L.ordfirst[o] = pre;
              L.upos[u] = (uint16_t)pre;
            }
            carry += tot;
          }
          wave_sync();
          // ---- scatter ids (sentence s's ids start at sent_off[s]-base) ----
          for (int u = lane; u < nunits; u += 64) {
            const int o = L.nord[L.ustart[u]];
            const int c = L.ucnt[u];
            const int32_t t0 = (o == 0 ? stok : 0) + (L.upos[u] - L.ordfirst[o]);
            const int64_t ob = (o == 0 ? P.sent_off[sc] : L.sst[o - 1]) - base;
            const int st0 = L.ustage[u];
            for (int q = 0; q < c; ++q)
              if (t0 + q < P.max_tok) P.out_ids[ob + t0 + q] = L.stage[lane][st0 + q];
          }
          STAMP(6);
          // ---- sentences that ended inside the window ----------------------
          const int on = ordinal_of(L, cur_new);
          if (lane < on) P.out_ntok[sc + lane] = min((lane == 0 ? stok : 0) + L.ordcnt[lane], P.max_tok);
          const int32_t stok_new = (on == 0 ? stok : 0) + L.ordcnt[on];
          wave_sync();
          stok = stok_new;
          cur = cur_new;
          if (on > 0) {
            sc += on;
            load_sst(L, P, sc, s_hi, lane);
          }
          wave_sync();
          STAMP(7);
          continue;
        }
      }
      if (dbg && lane == 0) atomicAdd((unsigned long long*)&P.dbg[13], 1ull);
      // ---- serial fallback: the rest of sentence sc on lane 0 (exact) -----
      wave_sync();
      const int64_t sc_end = L.sst[0];
      if (lane == 0) {
        SentState st{cur, sc_end, P.sent_off[sc] - base, stok};
        while (st.p < st.e && st.ntok < P.max_tok) step(P, st, fb, ascii_tab);
        P.out_ntok[sc] = min(st.ntok, P.max_tok);
      }
      cur = sc_end;
      stok = 0;
      sc += 1;
      wave_sync();
      load_sst(L, P, sc, s_hi, lane);
      wave_sync();
    }
  }
  if (dbg && lane == 0)
    for (int k = 0; k < 11; ++k) atomicAdd((unsigned long long*)&P.dbg[k], (unsigned long long)acc[k]);
#undef STAMP
}

const void* tokenize_kernel_ptr() { return reinterpret_cast<const void*>(&tokenize_kernel); }
const void* tokenize_wave_kernel_ptr() { return reinterpret_cast<const void*>(&tokenize_wave_kernel); }

hipError_t launch_tokenize(const TokParams& P, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(tokenize_kernel, dim3(grid), dim3(BLOCK), 0, stream, P);
  return hipGetLastError();
}

hipError_t launch_tokenize_wave(const TokParams& P, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(tokenize_wave_kernel, dim3(grid), dim3(64 * TOK_WAVES), 0, stream, P);
  return hipGetLastError();
}

}  // namespace lddl
