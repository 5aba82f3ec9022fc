// Pair packing (BERT NSP, CodeBERT doc/code segments), partition shuffle,
// sequence binning and row materialisation for gfx950.
//
// Reference:
//   BERT      lddl/dask/bert/pretrain.py:241-365 create_pairs_from_document,
//             :161-176 _truncate_seq_pair, :386-402 _to_partition_pairs
//   CodeBERT  lddl/dask/bert/pretrain_codebert.py:343-442, :236-247, :460-477
//   binning   lddl/dask/bert/binning.py:63-93 _to_dataframe_binned
//             (bin = (num_tokens-1)//bin_size clamped, stable per-bin order)
// Restated on the CPU in oracle/pack_oracle.py.
//
// Partition p (docs [part_doc_off[p], part_doc_off[p+1])) is the unit of
// independence: the random-next document is drawn from the same partition
// and the RNG stream (CPython MT19937 seeded with seed + p) is serial within
// it.  The packers (one wave per partition) are in pack_wave.hip; this file
// holds the partition scans, materialisation (the bulk byte work: gathering
// token ids into [CLS] A [SEP] B [SEP] rows, wave-parallel per 64 rows), the
// token offset scans and the static-masking kernels.
#include <algorithm>

#include "common.h"
#include "pack.h"
#include "wave.h"

namespace lddl {

// ------------------------------------------------- partition scans ----
// exclusive scans of two int64 arrays (n entries) into n+1 entries, one block
__global__ __launch_bounds__(1024) void scan_parts_kernel(const int64_t* a, const int64_t* b, int64_t n,
                                                          int64_t* sa, int64_t* sb, const int32_t* err,
                                                          int32_t* err_any) {
  __shared__ int64_t la[1024], lb[1024];
  __shared__ int32_t le;
  const int t = threadIdx.x;
  const int64_t per = (n + 1023) / 1024;
  const int64_t lo = min(n, t * per), hi = min(n, lo + per);
  int64_t x = 0, y = 0;
  int32_t e = 0;
  for (int64_t i = lo; i < hi; ++i) { x += a[i]; y += b[i]; e |= err[i]; }
  la[t] = x; lb[t] = y;
  if (t == 0) le = 0;
  __syncthreads();
  if (e) atomicOr(&le, e);
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive
    int64_t u = t >= off ? la[t - off] : 0, w = t >= off ? lb[t - off] : 0;
    __syncthreads();
    la[t] += u; lb[t] += w;
    __syncthreads();
  }
  int64_t ra = la[t] - x, rb = lb[t] - y;
  for (int64_t i = lo; i < hi; ++i) { sa[i] = ra; sb[i] = rb; ra += a[i]; rb += b[i]; }
  if (t == 1023) { sa[n] = la[1023]; sb[n] = lb[1023]; *err_any = le; }
}

// ----------------------------------------------------- materialise ----
// A segment is n consecutive filtered sentences cut to [lo, hi); in the dense
// id array (sentences' ids back to back) that is ONE run starting at
// fs_dense[fs] + lo.  One wave per partition (no row -> partition search):
// chunks of 64 rows are staged in LDS (record, offsets, runs), then copied by
// half-waves, one row each, 16 tokens per lane in flight.
struct RowStage {
  int64_t off;        // first output token of the row
  int64_t src0, src1; // dense offsets of segment 0 / 1
  int32_t l0, l1;     // segment lengths
  int32_t nt;         // num_tokens
  int32_t seg0;       // [SEP] after segment 0
};

__global__ __launch_bounds__(256) void materialize_kernel(MatParams M) {
  __shared__ RowStage st[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t total = M.pair_base[M.n_part];
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t p = (int64_t)blockIdx.x * 4 + wv; p < M.n_part; p += nw) {
    const int64_t s0 = M.doc_sent_off[M.part_doc_off[p]];
    const int64_t pb = (int64_t)M.dup * s0;
    const int64_t g0 = M.pair_base[p], np = M.pair_base[p + 1] - g0, tb = M.tok_base[p];
    for (int64_t c = 0; c < np; c += 64) {
      const int64_t i = c + lane;
      if (i < np) {
        const PairRec r = M.pairs[pb + M.binned[pb + i]];
        const int64_t off = tb + M.tok_local[pb + i];
        const int32_t l0 = r.hi0 - r.lo0, l1 = r.hi1 - r.lo1;
        const int64_t g = g0 + i;
        RowStage& x = st[wv][lane];
        x.off = off;
        x.src0 = l0 > 0 ? M.fs_dense[r.fs0] + r.lo0 : 0;
        x.src1 = l1 > 0 ? M.fs_dense[r.fs1] + r.lo1 : 0;
        x.l0 = l0;
        x.l1 = l1;
        x.nt = r.num_tokens;
        x.seg0 = (r.flags & 2) != 0;
        M.out_tok_off[g] = off;
        M.out_len0[g] = (uint16_t)l0;
        M.out_len1[g] = (uint16_t)l1;
        M.out_flags[g] = (uint8_t)r.flags;
        const int32_t b = ((int32_t)r.num_tokens - 1) / M.bin_size;
        M.out_bin[g] = (uint8_t)(b > M.nbins - 1 ? M.nbins - 1 : b);
        M.out_part[g] = p;
        if (g == total - 1) M.out_tok_off[total] = off + r.num_tokens;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int nr = (int)min((int64_t)64, np - c);
      const int hl = lane & 31;
      for (int r0 = 0; r0 < nr; r0 += 2) {
        const int rr = r0 + (lane >> 5);
        if (rr >= nr) continue;
        const RowStage x = st[wv][rr];
        uint16_t* out = M.out_tokens + x.off;
        const int b1 = 1 + x.l0 + x.seg0;  // first token of segment 1
        for (int t0 = 0; t0 < x.nt; t0 += 512) {
          uint16_t v[16];
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            const int t = t0 + hl + 32 * k;
            uint16_t y = (uint16_t)M.sep_id;
            if (t == 0) y = (uint16_t)M.cls_id;
            else if (t <= x.l0) y = M.dense[x.src0 + (t - 1)];
            else if (t >= b1 && t < b1 + x.l1) y = M.dense[x.src1 + (t - b1)];
            v[k] = y;
          }
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            const int t = t0 + hl + 32 * k;
            if (t < x.nt) out[t] = v[k];
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
}

// ---- chunked row copy (materialize v2) --------------------------------------
// A wave owns 64 consecutive rows whose outputs form one contiguous range
// [G0, G1); a row is [CLS] A [SEP] (B [SEP]) from the tokenizer's dense ids.
// Waves are dispatched in
// row order, so the resident waves touch only a narrow window of the source
// (the dup-fold re-reads of a sentence's ids in materialize stay on-die).
// The range is written in aligned 8-token (16-B) chunks.  Phase 1 is
// branch-free, MAT_U chunks per lane in flight: a chunk inside one source
// segment is two aligned 16-B loads funnel-shifted into one 16-B store.
// Every other chunk ([CLS]/[SEP], a row boundary, or one of the two chunks
// shared with the neighbouring waves) goes to a per-wave list that phase 2
// drains token-parallel (one token per lane, u16 load + store).
constexpr int MAT_U = 2;         // chunks per lane per phase-1 iteration (1 / 3 within noise, 8 slower)
constexpr int MAT_SLOW = 512;    // slow-chunk list capacity per wave
constexpr int MAT_PBITS = 26;    // slow entry: chunk start + 8 (26 bits) | row << 26
struct RowDesc {
  int64_t src0, src1;       // source start of segment A / B
  int32_t l0, b1, l1, nt;   // |A|, first position of B, |B|, row length
};
struct MatWave {
  int32_t roff[64];         // row start relative to G0 (INT_MAX past the last row)
  RowDesc row[64];
  uint32_t slow[MAT_SLOW];
};

// u16 window [m, m + 8) of the 16 u16 held in A:B
__device__ __forceinline__ uint4 funnel8(const uint4 A, const uint4 B, uint32_t m) {
  const uint32_t h = m >> 1, sh = (m & 1u) * 16u;
  const bool h0 = h == 0, h1 = h == 1, h2 = h == 2;
  const uint32_t e0 = h0 ? A.x : h1 ? A.y : h2 ? A.z : A.w;
  const uint32_t e1 = h0 ? A.y : h1 ? A.z : h2 ? A.w : B.x;
  const uint32_t e2 = h0 ? A.z : h1 ? A.w : h2 ? B.x : B.y;
  const uint32_t e3 = h0 ? A.w : h1 ? B.x : h2 ? B.y : B.z;
  const uint32_t e4 = h0 ? B.x : h1 ? B.y : h2 ? B.z : B.w;
  return make_uint4(__builtin_amdgcn_alignbit(e1, e0, sh), __builtin_amdgcn_alignbit(e2, e1, sh),
                    __builtin_amdgcn_alignbit(e3, e2, sh), __builtin_amdgcn_alignbit(e4, e3, sh));
}

__device__ __forceinline__ void mat_wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// last row starting at or before p (rows may be empty: the last of equals)
__device__ __forceinline__ int mat_row(const MatWave& W, int32_t p) {
  int r = 0;
#pragma unroll
  for (int st = 32; st >= 1; st >>= 1)
    if (W.roff[r + st] <= p) r += st;
  return r;
}

// token t of row x: the special it is (false) or its source index (true)
__device__ __forceinline__ bool mat_tok(const RowDesc& x, int32_t t, uint32_t cls, uint32_t& y, int64_t& src) {
  if (t == 0) { y = cls; return false; }
  if (t <= x.l0) { src = x.src0 + (t - 1); return true; }
  if (t >= x.b1 && t < x.b1 + x.l1) { src = x.src1 + (t - x.b1); return true; }
  return false;  // [SEP]
}

// phase 2: tokens [0, ntok) of the listed chunks (or, with W == nullptr
// semantics via plain, every position of the range), one token per lane
__device__ __forceinline__ void mat_drain(const MatWave& W, int ntok, bool listed, int64_t G0, int32_t G1r,
                                          const uint16_t* src, uint16_t* out, uint32_t cls, uint32_t sep,
                                          int lane) {
  mat_wsync();
  for (int j0 = 0; j0 < ntok; j0 += 4 * 64) {
    uint32_t y[4];
    int32_t pos[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int j = j0 + m * 64 + lane;
      pos[m] = -1;
      y[m] = sep;
      int64_t s = 0;
      bool ld = false;
      if (j < ntok) {
        const int32_t p = listed ? (int32_t)(W.slow[j >> 3] & ((1u << MAT_PBITS) - 1u)) - 8 + (j & 7) : j;
        if (p >= 0 && p < G1r) {
          const int r = mat_row(W, p);
          pos[m] = p;
          ld = mat_tok(W.row[r], p - W.roff[r], cls, y[m], s);
        }
      }
      if (ld) y[m] = src[s];
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
      if (pos[m] >= 0) out[G0 + pos[m]] = (uint16_t)y[m];
  }
  mat_wsync();
}

// rows published in W (roff, row) for nr rows spanning [G0, G1) of out;
// src readable for n_src entries
__device__ __forceinline__ void mat_copy(MatWave& W, int64_t G0, int64_t G1, const uint16_t* src, int64_t n_src,
                                         uint16_t* out, uint32_t cls, uint32_t sep, int lane) {
  const int32_t G1r = (int32_t)(G1 - G0);
  if (G1 - G0 >= (1 << MAT_PBITS) - 16) {  // (rows beyond any real max_tok) token by token
    mat_drain(W, G1r, false, G0, G1r, src, out, cls, sep, lane);
    return;
  }
  const int64_t q0 = G0 >> 3, q1 = (G1 + 7) >> 3;
  uint4* out4 = reinterpret_cast<uint4*>(out);
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  const int64_t amax = (n_src >> 3) - 2;  // last 16-B pair fully inside src
  int ns = 0;  // listed slow chunks (wave-uniform)
  for (int64_t qb = q0; qb < q1; qb += MAT_U * 64) {
    int64_t sv[MAT_U];
    bool fast[MAT_U], slow[MAT_U];
    int rw[MAT_U];
#pragma unroll
    for (int u = 0; u < MAT_U; ++u) {
      const int64_t q = qb + u * 64 + lane;
      const int32_t p0 = (int32_t)((q << 3) - G0);
      const int r = mat_row(W, p0 < 0 ? 0 : p0);
      rw[u] = r;
      const RowDesc y = W.row[r];
      const int32_t t0 = p0 - W.roff[r];
      bool inA, inB;
      int64_t v;
      inA = t0 >= 1 && t0 + 8 <= 1 + y.l0;
      inB = t0 >= y.b1 && t0 + 8 <= y.b1 + y.l1;
      v = inA ? y.src0 + (t0 - 1) : y.src1 + (t0 - y.b1);
      fast[u] = q < q1 && (inA || inB) && (v >> 3) <= amax;
      slow[u] = q < q1 && !fast[u];
      sv[u] = fast[u] ? v : 0;
    }
    uint4 va[MAT_U], vb[MAT_U];
#pragma unroll
    for (int u = 0; u < MAT_U; ++u) {
      const int64_t a = sv[u] >> 3;
      va[u] = vb[u] = make_uint4(0, 0, 0, 0);
      if (fast[u]) {  // exec-masked: no load past a short source
        va[u] = s4[a];
        vb[u] = s4[a + 1];
      }
    }
#pragma unroll
    for (int u = 0; u < MAT_U; ++u)
      if (fast[u]) {
        const uint4 v = funnel8(va[u], vb[u], (uint32_t)(sv[u] & 7));
        // the packed rows are written once and read next by the host copy:
        // streaming stores keep L2 for the dup-fold re-reads of the dense ids
        // (materialize 28.3 -> 25.0 ms)
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        u32x4 w;
        w.x = v.x; w.y = v.y; w.z = v.z; w.w = v.w;
        __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(out4) + (qb + u * 64 + lane));
      }
#pragma unroll
    for (int u = 0; u < MAT_U; ++u) {
      const uint64_t m = __ballot(slow[u]);
      if (slow[u]) {
        const int32_t p0 = (int32_t)(((qb + u * 64 + lane) << 3) - G0);
        W.slow[ns + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)(p0 + 8) | ((uint32_t)rw[u] << MAT_PBITS);
      }
      ns += __popcll(m);
    }
    if (ns > MAT_SLOW - MAT_U * 64) {
      mat_drain(W, ns * 8, true, G0, G1r, src, out, cls, sep, lane);
      ns = 0;
    }
  }
  if (ns > 0) mat_drain(W, ns * 8, true, G0, G1r, src, out, cls, sep, lane);
}

// workgroups are dealt round-robin to the 8 XCDs (one L2 each): block b runs
// on XCD b % 8, so map it to item range (b % 8) of 8 contiguous ranges --
// each XCD's L2 then holds the dense ids of a few partitions, not all of the
// ones in flight (the dup-fold re-reads hit L2 instead of the MALL / HBM)
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nblk) {
  if (nblk < 64) return b;
  const int64_t per = (nblk + 7) >> 3;
  return (b & 7) * per + (b >> 3);
}

__global__ __launch_bounds__(256) void materialize2_kernel(MatParams M, int64_t total, int64_t n_src) {
  __shared__ MatWave mw[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t gbase = (xcd_block(blockIdx.x, gridDim.x) * 4 + wv) * 64;
  if (gbase >= total) return;
  const int nr = (int)min((int64_t)64, total - gbase);
  MatWave& W = mw[wv];
  // partition of the item's first pair (uniform binary search over pair_base)
  int64_t plo = 0, phi = M.n_part - 1;
  while (plo < phi) {
    const int64_t mid = (plo + phi + 1) >> 1;
    if (M.pair_base[mid] <= gbase) plo = mid;
    else phi = mid - 1;
  }
  // ---- row metadata + per-pair outputs ----
  int64_t off = 0, rend = 0;
  RowDesc x{};
  if (lane < nr) {
    const int64_t g = gbase + lane;
    int64_t p = plo;
    while (M.pair_base[p + 1] <= g) ++p;  // partitions of < 64 pairs
    const int64_t i = g - M.pair_base[p];
    const int64_t pb = (int64_t)M.dup * M.doc_sent_off[M.part_doc_off[p]];
    const PairRec r = M.pairs[pb + M.binned[pb + i]];
    off = M.tok_base[p] + M.tok_local[pb + i];
    const int32_t l0 = r.hi0 - r.lo0, l1 = r.hi1 - r.lo1;
    x.src0 = l0 > 0 ? M.fs_dense[r.fs0] + r.lo0 : 0;
    x.src1 = l1 > 0 ? M.fs_dense[r.fs1] + r.lo1 : 0;
    x.l0 = l0;
    x.l1 = l1;
    x.b1 = 1 + l0 + ((r.flags & 2) != 0);
    x.nt = r.num_tokens;
    rend = off + r.num_tokens;
    M.out_tok_off[g] = off;
    M.out_len0[g] = (uint16_t)l0;
    M.out_len1[g] = (uint16_t)l1;
    M.out_flags[g] = (uint8_t)r.flags;
    const int32_t b = ((int32_t)r.num_tokens - 1) / M.bin_size;
    M.out_bin[g] = (uint8_t)(b > M.nbins - 1 ? M.nbins - 1 : b);
    M.out_part[g] = p;
    if (g == total - 1) M.out_tok_off[total] = rend;
  }
  const int64_t G0 = __shfl(off, 0), G1 = __shfl(rend, nr - 1);
  W.roff[lane] = lane < nr ? (int32_t)(off - G0) : 0x7FFFFFFF;
  W.row[lane] = x;
  mat_wsync();
  mat_copy(W, G0, G1, M.dense, n_src, M.out_tokens, M.cls_id, M.sep_id, lane);
}

#ifndef LDDL_ROWSPAN_XCD
#define LDDL_ROWSPAN_XCD 1
#endif
// Row spans (lddl_row_spans): the rows of materialize2 without the token
// copy.  Each segment of a row is ONE contiguous run of the tokenizer's dense
// ids (a document's sentences are contiguous there and a segment is a window
// of consecutive sentences), so row g = [CLS] ids[src0, src0 + len0) [SEP]
// ids[src1, src1 + len1) [SEP] is fully described by two offsets; the string
// columns (lddl_render_strings, RENDER_SPAN) and the loaders read the ids
// through them.  Wave per 64 rows, lane per row: the same metadata chain as
// materialize2 (partition, binned record, pair record, segment starts) and
// ~38 B written per row instead of the row's 2 B per token.
// Per partition p: part_pb[p] and the 64-row chunks whose first row is p's
// (chunk_part), so a row-spans wave finds its partition with one load instead
// of a binary search over pair_base (15 dependent loads per wave).
__global__ __launch_bounds__(256) void chunk_parts_kernel(const int64_t* pair_base, const int64_t* doc_sent_off,
                                                          const int64_t* part_doc_off, int32_t dup, int64_t n_part,
                                                          int32_t* chunk_part, int64_t* part_pb) {
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < n_part; p += (int64_t)gridDim.x * 256) {
    part_pb[p] = (int64_t)dup * doc_sent_off[part_doc_off[p]];
    const int64_t c0 = (pair_base[p] + 63) >> 6, c1 = (pair_base[p + 1] + 63) >> 6;
    for (int64_t c = c0; c < c1; ++c) chunk_part[c] = (int32_t)p;
  }
}

hipError_t launch_chunk_parts(const int64_t* pair_base, const int64_t* doc_sent_off, const int64_t* part_doc_off,
                              int32_t dup, int64_t n_part, int32_t* chunk_part, int64_t* part_pb, hipStream_t s) {
  const int64_t nblk = std::max<int64_t>(1, std::min<int64_t>((n_part + 255) / 256, 1024));
  hipLaunchKernelGGL(chunk_parts_kernel, dim3((unsigned)nblk), dim3(256), 0, s, pair_base, doc_sent_off, part_doc_off,
                     dup, n_part, chunk_part, part_pb);
  return hipGetLastError();
}

// (XCD-aware blocks, as materialize2: a partition's rows run on one XCD, so
// its pair records and binned order are fetched into one L2, not all eight)
// RS_U consecutive 64-row chunks per wave, each metadata level loaded for all
// of them before the next: a row's chain (partition -> bases -> binned
// index -> pair record -> segment offsets) is ~6 dependent loads, and
// RS_U chains in flight per wave instead of one
#ifndef LDDL_ROWSPAN_U
#define LDDL_ROWSPAN_U 2
#endif
constexpr int RS_U = LDDL_ROWSPAN_U;
__global__ __launch_bounds__(256) void rowspan_kernel(MatParams M, int64_t total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t gbase =
      (LDDL_ROWSPAN_XCD ? xcd_block(blockIdx.x, gridDim.x) * 4 + wv : (int64_t)blockIdx.x * 4 + wv) * 64 * RS_U;
  if (gbase >= total) return;
  int64_t g[RS_U], p[RS_U];
  bool in[RS_U];
#pragma unroll
  for (int u = 0; u < RS_U; ++u) {
    g[u] = gbase + 64 * u + lane;
    in[u] = g[u] < total;
    p[u] = in[u] ? M.chunk_part[(gbase >> 6) + u] : 0;
  }
  int64_t i[RS_U], pb[RS_U];
#pragma unroll
  for (int u = 0; u < RS_U; ++u) {
    if (in[u]) {
      while (M.pair_base[p[u] + 1] <= g[u]) ++p[u];  // partitions of < 64 pairs
    }
    i[u] = in[u] ? g[u] - M.pair_base[p[u]] : 0;
    pb[u] = in[u] ? M.part_pb[p[u]] : 0;
  }
  int32_t bi[RS_U];
#pragma unroll
  for (int u = 0; u < RS_U; ++u) bi[u] = in[u] ? M.binned[pb[u] + i[u]] : 0;
  PairRec r[RS_U];
#pragma unroll
  for (int u = 0; u < RS_U; ++u) r[u] = M.pairs[in[u] ? pb[u] + bi[u] : 0];
#pragma unroll
  for (int u = 0; u < RS_U; ++u) {
    if (!in[u]) continue;
    const int32_t l0 = r[u].hi0 - r[u].lo0, l1 = r[u].hi1 - r[u].lo1;
    M.out_src0[g[u]] = l0 > 0 ? M.fs_dense[r[u].fs0] + r[u].lo0 : 0;
    M.out_src1[g[u]] = l1 > 0 ? M.fs_dense[r[u].fs1] + r[u].lo1 : 0;
    if (M.out_tok_off) {
      const int64_t off = M.tok_base[p[u]] + M.tok_local[pb[u] + i[u]];
      M.out_tok_off[g[u]] = off;
      if (g[u] == total - 1) M.out_tok_off[total] = off + r[u].num_tokens;
    }
    M.out_len0[g[u]] = (uint16_t)l0;
    M.out_len1[g[u]] = (uint16_t)l1;
    M.out_flags[g[u]] = (uint8_t)r[u].flags;
    const int32_t bb = ((int32_t)r[u].num_tokens - 1) / M.bin_size;
    M.out_bin[g[u]] = (uint8_t)(bb > M.nbins - 1 ? M.nbins - 1 : bb);
    M.out_part[g[u]] = p[u];
  }
}

hipError_t launch_row_spans(const MatParams& M, int64_t total_pairs, hipStream_t s) {
  int64_t nblk = (total_pairs + 256 * RS_U - 1) / (256 * RS_U);
  if (LDDL_ROWSPAN_XCD && nblk >= 64) nblk = (nblk + 7) & ~(int64_t)7;  // xcd_block: 8 equal ranges (extra blocks exit)
  hipLaunchKernelGGL(rowspan_kernel, dim3((unsigned)nblk), dim3(256), 0, s, M, total_pairs);
  return hipGetLastError();
}

// ------------------------------------------------- token offset scans ----
constexpr int SCAN_ITEMS = 4096;  // ntok entries per scan block (256 x 16)

__host__ __device__ int64_t scan_blocks(int64_t n) { return (n + SCAN_ITEMS - 1) / SCAN_ITEMS; }

__device__ __forceinline__ int64_t block_excl_scan256(int64_t v, int64_t* red, int64_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) red[w] = x;
  __syncthreads();
  int64_t pre = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k < w) pre += red[k];
    tot += red[k];
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

// The scan's range [lo, hi) comes from the device (d_lo / d_hi, e.g. a
// tokenizer segment's sentences) or is [0, n) (d_lo == nullptr); the grid is
// sized for at most n items and blocks past the range exit.  With d_lo, the
// scan continues from tokoff[lo] (the previous range's total).
__device__ __forceinline__ void scan_range(const int64_t* d_lo, const int64_t* d_hi, int64_t n, int64_t& lo,
                                           int64_t& hi) {
  lo = d_lo ? *d_lo : 0;
  hi = d_lo ? *d_hi : n;
}

__global__ __launch_bounds__(256) void scan_reduce_kernel(const int32_t* ntok, const int64_t* d_lo, const int64_t* d_hi,
                                                          int64_t n, int64_t* bsum) {
  __shared__ int64_t red[4];
  int64_t lo, hi;
  scan_range(d_lo, d_hi, n, lo, hi);
  const int64_t b0 = lo + (int64_t)blockIdx.x * SCAN_ITEMS;
  if (b0 >= hi) return;
  int64_t sum = 0;
  for (int k = threadIdx.x; k < SCAN_ITEMS; k += 256)
    if (b0 + k < hi) sum += ntok[b0 + k];
  int64_t tot;
  block_excl_scan256(sum, red, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// exclusive scan of the block sums in place (one block), bsum[nb] = total
__global__ __launch_bounds__(256) void scan_bsum_kernel(int64_t* bsum, const int64_t* d_lo, const int64_t* d_hi,
                                                        int64_t n, const int64_t* tokoff) {
  __shared__ int64_t red[4];
  int64_t lo, hi;
  scan_range(d_lo, d_hi, n, lo, hi);
  const int64_t nb = scan_blocks(hi - lo);
  int64_t carry = d_lo ? tokoff[lo] : 0;
  for (int64_t c = 0; c < nb; c += 256) {
    const int64_t i = c + threadIdx.x;
    const int64_t v = i < nb ? bsum[i] : 0;
    int64_t tot;
    const int64_t ex = block_excl_scan256(v, red, &tot);
    if (i < nb) bsum[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) bsum[nb] = carry;
}

__global__ __launch_bounds__(256) void scan_write_kernel(const int32_t* ntok, const int64_t* d_lo, const int64_t* d_hi,
                                                         int64_t n, const int64_t* bsum, int64_t* tokoff) {
  __shared__ int64_t red[4];
  int64_t lo, hi;
  scan_range(d_lo, d_hi, n, lo, hi);
  if (lo + (int64_t)blockIdx.x * SCAN_ITEMS >= hi) return;
  const int64_t b0 = lo + (int64_t)blockIdx.x * SCAN_ITEMS + threadIdx.x * 16;
  int32_t v[16];
  int64_t sum = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    v[k] = b0 + k < hi ? ntok[b0 + k] : 0;
    sum += v[k];
  }
  int64_t tot;
  int64_t run = bsum[blockIdx.x] + block_excl_scan256(sum, red, &tot);
  // the offsets go out through LDS so that consecutive lanes store
  // consecutive offsets (a thread's 16 offsets stored directly put 64 lines
  // under every store instruction); one pad slot per 16 spreads the
  // thread-major writes over the banks
  __shared__ int64_t ob[SCAN_ITEMS + SCAN_ITEMS / 16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    ob[threadIdx.x * 17 + k] = run;
    run += v[k];
  }
  __syncthreads();
  const int64_t c0 = lo + (int64_t)blockIdx.x * SCAN_ITEMS;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int j = k * 256 + threadIdx.x;
    if (c0 + j < hi) tokoff[c0 + j] = ob[j + (j >> 4)];
  }
  if (lo + ((int64_t)blockIdx.x + 1) * SCAN_ITEMS >= hi && threadIdx.x == 0) tokoff[hi] = bsum[scan_blocks(hi - lo)];
}

static hipError_t scan_launch(const int32_t* ntok, const int64_t* d_lo, const int64_t* d_hi, int64_t n,
                              int64_t* tokoff, int64_t* blocksums, hipStream_t s) {
  const int64_t nb = scan_blocks(n);
  if (nb == 0) return d_lo ? hipSuccess : hipMemsetAsync(tokoff, 0, sizeof(int64_t), s);
  hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nb), dim3(256), 0, s, ntok, d_lo, d_hi, n, blocksums);
  hipLaunchKernelGGL(scan_bsum_kernel, dim3(1), dim3(256), 0, s, blocksums, d_lo, d_hi, n, (const int64_t*)tokoff);
  hipLaunchKernelGGL(scan_write_kernel, dim3((unsigned)nb), dim3(256), 0, s, ntok, d_lo, d_hi, n,
                     (const int64_t*)blocksums, tokoff);
  return hipGetLastError();
}

hipError_t launch_scan_ntok(const int32_t* ntok, int64_t n, int64_t* tokoff, int64_t* blocksums, hipStream_t s) {
  return scan_launch(ntok, nullptr, nullptr, n, tokoff, blocksums, s);
}

hipError_t launch_scan_ntok_range(const int32_t* ntok, const int64_t* d_lo, const int64_t* d_hi, int64_t max_items,
                                  int64_t* tokoff, int64_t* blocksums, hipStream_t s) {
  return scan_launch(ntok, d_lo, d_hi, max_items, tokoff, blocksums, s);
}

hipError_t launch_scan_parts(const int64_t* a, const int64_t* b, int64_t n, int64_t* sa, int64_t* sb,
                             const int32_t* err, int32_t* err_any, hipStream_t s) {
  hipLaunchKernelGGL(scan_parts_kernel, dim3(1), dim3(1024), 0, s, a, b, n, sa, sb, err, err_any);
  return hipGetLastError();
}

// ----------------------------------------------------- static masking ----
// sentence s holds a token equal to [CLS] or [SEP] (literal special tokens in
// the text): create_masked_lm_predictions excludes those from the candidates
// (pretrain.py:187-190), so pairs touching such a sentence build an explicit
// candidate list; all others use the implicit one.
__global__ __launch_bounds__(256) void sent_special_kernel(const uint16_t* ids, const int64_t* tok_off,
                                                           const int32_t* ntok, int64_t n_sent, uint32_t cls,
                                                           uint32_t sep, uint8_t* out) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_sent; s += (int64_t)gridDim.x * blockDim.x) {
    const uint16_t* t = ids + tok_off[s];
    const int n = ntok[s];
    uint32_t f = 0;
    for (int k = 0; k < n; ++k) {
      const uint32_t v = t[k];
      f |= (v == cls) | (v == sep);
    }
    out[s] = (uint8_t)f;
  }
}

// Row g of the materialised output: copy its masked entries (sorted by
// position, pretrain.py:225) to the global position/label lists and apply the
// replacement in place.  label = the row's token before replacement.
// Four rows per wave (16 lanes each): a row's metadata is a chain of
// dependent loads (partition -> its bases -> binned record -> masking ref),
// so the wave keeps four chains in flight.
__global__ __launch_bounds__(256) void masked_lm_kernel(MlmParams M) {
  const int sl = threadIdx.x & 15;
  const int64_t total = M.pair_base[M.n_part];
  const int64_t ng = (int64_t)gridDim.x * 16;  // row groups of 16 lanes
  for (int64_t g = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4); g < total; g += ng) {
    const int64_t p = M.row_part[g];  // (materialize wrote every row's partition)
    const int64_t i = g - M.pair_base[p];
    const int64_t pb = (int64_t)M.dup * M.doc_sent_off[M.part_doc_off[p]];
    const int64_t ref = M.mref[pb + M.binned[pb + i]];
    const int nm = (int)((uint64_t)ref >> 48);
    const int64_t aoff = ref & ((int64_t(1) << 48) - 1);
    const int64_t ooff = M.mask_base[p] + M.mloc[pb + i];
    uint16_t* row = M.tokens + M.tok_off[g];
    if (sl == 0) {
      M.out_off[g] = ooff;
      if (g == total - 1) M.out_off[total] = ooff + nm;
    }
    for (int k = sl; k < nm; k += 16) {
      const uint32_t e = M.marena[aoff + k];
      const uint32_t pos = e & 0xFFFFu, nid = e >> 16;
      const uint16_t label = row[pos];
      M.out_pos[ooff + k] = (uint16_t)pos;
      M.out_label[ooff + k] = label;
      if (nid != MLM_KEEP) row[pos] = (uint16_t)nid;
    }
  }
}

// The same over rows described by spans (lddl_row_spans): no row to mask in
// place; a masked position's label is read from the dense ids through the
// row's span (A = positions 1 .. len0, [SEP], B from len0 + 2: candidates
// never include [CLS] / [SEP], pretrain.py:187-190) and the token the masked
// row shows there (the replacement, or the label when kept) goes to
// out_token for the writer (lddl_render_masked).
constexpr int MLM_SPAN_UNROLL = 8;  // masked positions per lane with loads in flight together

__global__ __launch_bounds__(256) void masked_lm_spans_kernel(MlmParams M) {
  // A wave per 64 rows.  First every lane resolves one row (partition, its
  // pair's arena reference, output offset, span starts): the rows' dependent
  // lookups are all in flight together instead of one row per 16 lanes at a
  // time.  Then the 64 rows' masked positions are walked as one flat list,
  // MLM_SPAN_UNROLL positions per lane at a time (their arena and id loads in
  // flight together); a position's row is found by advancing a per-lane row
  // cursor over the rows' exclusive position counts in LDS, and the outputs
  // of consecutive positions are adjacent (coalesced stores).
  struct RowLds {
    int64_t aoff[64], ooff[64], a[64], b[64];
    int32_t l0[64], pre[65];
  };
  __shared__ RowLds R[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  RowLds& L = R[wv];
  const int64_t total = M.pair_base[M.n_part];
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t g0 = ((int64_t)blockIdx.x * 4 + wv) * 64; g0 < total; g0 += nw * 64) {
    const int64_t g = g0 + lane;
    int nm = 0;
    if (g < total) {
      const int64_t p = M.row_part[g];
      const int64_t i = g - M.pair_base[p];
      const int64_t pb = (int64_t)M.dup * M.doc_sent_off[M.part_doc_off[p]];
      const int64_t ref = M.mref[pb + M.binned[pb + i]];
      nm = (int)((uint64_t)ref >> 48);
      const int64_t ooff = M.mask_base[p] + M.mloc[pb + i];
      L.aoff[lane] = ref & ((int64_t(1) << 48) - 1);
      L.ooff[lane] = ooff;
      L.a[lane] = M.src0[g];
      L.b[lane] = M.src1[g];
      L.l0[lane] = M.len0[g];
      M.out_off[g] = ooff;
      if (g == total - 1) M.out_off[total] = ooff + nm;
    }
    const int incl = wave_incl_add(nm);
    L.pre[lane] = incl - nm;
    if (lane == 63) L.pre[64] = incl;
    const int T = lane_get(incl, 63);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int r = 0;  // this lane's row cursor (positions rise with t)
    constexpr int U = MLM_SPAN_UNROLL;
    for (int t0 = 0; t0 < T; t0 += 64 * U) {
      int rr[U], kk[U];
      uint32_t e[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int t = t0 + 64 * u + lane;
        rr[u] = -1;
        if (t < T) {
          while (L.pre[r + 1] <= t) ++r;
          rr[u] = r;
          kk[u] = t - L.pre[r];
          e[u] = M.marena[L.aoff[r] + kk[u]];
        }
      }
      uint16_t lab[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (rr[u] >= 0) {
          const int q = rr[u];
          const int32_t pos = (int32_t)(e[u] & 0xFFFFu);
          lab[u] = M.ids[pos <= L.l0[q] ? L.a[q] + (pos - 1) : L.b[q] + (pos - L.l0[q] - 2)];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (rr[u] >= 0) {
          const int q = rr[u];
          const int64_t o = L.ooff[q] + kk[u];
          const uint32_t nid = e[u] >> 16;
          M.out_pos[o] = (uint16_t)(e[u] & 0xFFFFu);
          M.out_label[o] = lab[u];
          M.out_token[o] = nid != MLM_KEEP ? (uint16_t)nid : lab[u];
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

hipError_t launch_sent_special(const uint16_t* ids, const int64_t* tok_off, const int32_t* ntok, int64_t n_sent,
                               uint32_t cls, uint32_t sep, uint8_t* out, hipStream_t s) {
  hipLaunchKernelGGL(sent_special_kernel, dim3(4096), dim3(256), 0, s, ids, tok_off, ntok, n_sent, cls, sep, out);
  return hipGetLastError();
}

// masked_lm_spans_kernel's grid: up to one 64-row group per wave (blocks of 4
// waves), capped at LDDL_MLM_GRID blocks -- the hardware then balances the
// launch instead of a fixed grid-stride share per wave (4096 blocks: 424.5,
// 65 536: 420.8 ms per masked step, profiles/r6/v/)
#ifndef LDDL_MLM_GRID
#define LDDL_MLM_GRID (1 << 20)
#endif
hipError_t launch_masked_lm(const MlmParams& M, int64_t n_rows, hipStream_t s) {
  if (M.tokens) {
    hipLaunchKernelGGL(masked_lm_kernel, dim3(2048), dim3(256), 0, s, M);
  } else {
    const int64_t grid = std::max<int64_t>(1, std::min<int64_t>((n_rows + 255) / 256, LDDL_MLM_GRID));
    hipLaunchKernelGGL(masked_lm_spans_kernel, dim3((unsigned)grid), dim3(256), 0, s, M);
  }
  return hipGetLastError();
}

hipError_t launch_materialize(const MatParams& M, int64_t total_pairs, int64_t n_dense, int algo, hipStream_t s) {
  // v2 needs 16-B aligned output and dense ids
  if (algo != 1 && ((reinterpret_cast<uintptr_t>(M.out_tokens) | reinterpret_cast<uintptr_t>(M.dense)) & 15u) == 0) {
    const int64_t items = (total_pairs + 63) / 64;  // one wave per 64 pairs
    int64_t nblk = (items + 3) / 4;
    if (nblk >= 64) nblk = (nblk + 7) & ~(int64_t)7;  // xcd_block: 8 equal ranges (extra blocks exit)
    hipLaunchKernelGGL(materialize2_kernel, dim3((unsigned)nblk), dim3(256), 0, s, M, total_pairs, n_dense);
  } else {
    const int64_t grid = (M.n_part + 3) / 4;  // one wave per partition
    hipLaunchKernelGGL(materialize_kernel, dim3((unsigned)grid), dim3(256), 0, s, M);
  }
  return hipGetLastError();
}

}  // namespace lddl
