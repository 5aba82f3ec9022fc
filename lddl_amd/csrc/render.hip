// String rendering of materialised rows (device side of lddl_render_strings /
// lddl_row_docs).
//
// The reference emits every packed instance as strings:
//   'A': ' '.join(tokens_a), 'B': ' '.join(tokens_b)            pretrain.py:348-353
//   'masked_lm_labels': ' '.join(masked_lm_labels)              pretrain.py:356-360
//   'id': document._id, 'doc': ' '.join(doc_tokens),
//   'code': ' '.join(code_tokens)                                pretrain_codebert.py:425-432
// and to_parquet stores them as Arrow string columns (int32 offsets + UTF-8
// bytes, pretrain.py:457-471).  Here a column is produced on the device in
// that layout: a per-row byte length, an exclusive scan into offsets, then
// the bytes -- ready for pa.StringArray.from_buffers after one D2H copy.
//
// Work mapping: one wave per row (rows are 2..1024 tokens; a seq-512 BERT
// row has ~370), 64 tokens per step.  Token strings come from a 4-aligned
// pool of the vocab entries (full text incl. "##", <= 200 KB, L2-resident);
// vinfo[id] = pool offset << 8 | length.  The bound is the output stream:
// per token ~6 B written against 2 B of id read.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "render.h"
#include "wave.h"

namespace lddl {

__device__ __forceinline__ void seg_of(const RenderParams& R, int64_t r, int64_t& start, int32_t& n) {
  const int64_t o = R.row_off[r];
  if (R.segment == RENDER_SPAN) {
    start = o;
    n = R.len0[r];
    return;
  }
  if (R.segment == RENDER_ROW) {
    start = o;
    n = (int32_t)(R.row_off[r + 1] - o);
    return;
  }
  const int32_t l0 = R.len0[r];
  if (R.segment == RENDER_SEG0) {
    start = o + 1;
    n = l0;
  } else {
    // [CLS] A [SEP] B [SEP]; CodeBERT: [CLS] code [SEP] when there is no doc
    // segment ([SEP] after seg0 only when flags bit1)
    const int32_t sep = R.codebert ? ((R.flags[r] >> 1) & 1) : 1;
    start = o + 1 + l0 + sep;
    n = R.len1[r];
  }
}

__device__ __forceinline__ void rwsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// token k0 + lane of row r's segment, with row r's masked positions applied
// (R.moff set): the row's patches falling in this chunk of 64 are scattered
// into the wave's LDS slots, then each lane reads its own
__device__ __forceinline__ uint32_t masked_tok(const RenderParams& R, uint32_t* pt, int64_t r, int32_t k0, int32_t n,
                                               int64_t start, int lane) {
  const int32_t k = k0 + lane;
  uint32_t id = k < n ? R.tokens[start + k] : 0u;
  if (!R.moff) return id;
  const int64_t m0 = R.moff[r], m1 = R.moff[r + 1];
  if (m0 == m1) return id;
  const int32_t base = (R.mseg == 0 ? 1 : (int32_t)R.len0m[r] + 2) + k0;
  rwsync();
  pt[lane] = 0u;
  rwsync();
  for (int64_t e = m0 + lane; e < m1; e += 64) {
    const int32_t rel = (int32_t)R.mpos[e] - base;
    if (rel >= 0 && rel < 64) pt[rel] = 0x10000u | R.mtok[e];
  }
  rwsync();
  const uint32_t v = pt[lane];
  return v ? (v & 0xFFFFu) : id;
}

// lens[r] = bytes of ' '.join(vocab[t] for t in segment(r))
__global__ __launch_bounds__(256) void render_len_kernel(RenderParams R) {
  __shared__ uint32_t ptch[4][64];
  const int lane = threadIdx.x & 63;
  uint32_t* const pt = ptch[threadIdx.x >> 6];
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < R.n_rows; i += nw) {
    int64_t start;
    int32_t n;
    seg_of(R, R.row0 + i, start, n);
    uint32_t acc = 0;
    for (int32_t k0 = 0; k0 < n; k0 += 64) {
      const uint32_t t = masked_tok(R, pt, R.row0 + i, k0, n, start, lane);
      if (k0 + lane < n) acc += (R.vinfo[t] & 0xFFu) + 1u;
    }
    // wave total: inclusive scan, lane 63 holds the sum
    acc = lane_get(wave_incl_add(acc), 63);
    if (lane == 0) R.lens[i] = n > 0 ? (int32_t)acc - 1 : 0;
  }
}

// bytes of row i at out[out_off[i] - out_off[0] ..]
__global__ __launch_bounds__(256) void render_bytes_kernel(RenderParams R) {
  __shared__ uint32_t ptch[4][64];
  const int lane = threadIdx.x & 63;
  uint32_t* const pt = ptch[threadIdx.x >> 6];
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t o0 = R.out_off[0];
  for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < R.n_rows; i += nw) {
    int64_t start;
    int32_t n;
    seg_of(R, R.row0 + i, start, n);
    int64_t base = R.out_off[i] - o0;
    for (int32_t k0 = 0; k0 < n; k0 += 64) {
      const int32_t k = k0 + lane;
      uint32_t info = 0, len = 0, w = 0;
      const uint32_t t = masked_tok(R, pt, R.row0 + i, k0, n, start, lane);
      if (k < n) {
        info = R.vinfo[t];
        len = info & 0xFFu;
        w = len + (k < n - 1 ? 1u : 0u);  // the joining space follows every token but the last
      }
      const uint32_t incl = wave_incl_add(w);
      if (k < n) {
        uint8_t* dst = R.out + base + (incl - w);
        const uint8_t* src = R.vpool + (info >> 8);
        for (uint32_t b = 0; b < len; ++b) dst[b] = src[b];
        if (w > len) dst[len] = ' ';
      }
      base += lane_get(incl, 63);
    }
  }
}

// Document of each row: the document holding the first sentence of the
// row's first non-empty segment.  Sentence by byte offset:
// the last s with sent_off[s] <= x (an empty sentence shares its offset with
// the next one, the last of such a run is the one holding x's bytes); then
// the last d with doc_sent_off[d] <= s.
__global__ __launch_bounds__(256) void row_docs_kernel(RowDocParams D) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < D.n_rows; g += stride) {
    int64_t plo = 0, phi = D.n_part - 1;
    while (plo < phi) {
      const int64_t mid = (plo + phi + 1) >> 1;
      if (D.pair_base[mid] <= g) plo = mid;
      else phi = mid - 1;
    }
    const int64_t p = plo;
    const int64_t pb = (int64_t)D.dup * D.doc_sent_off[D.part_doc_off[p]];
    const PairRec r = D.pairs[pb + D.binned[pb + (g - D.pair_base[p])]];
    // seg0 (A / doc) is the row's own document; a CodeBERT row without a doc
    // segment has only seg1 (BERT's B may come from a random document)
    const int64_t x = D.fs_base[r.hi0 > r.lo0 ? r.fs0 : r.fs1] + D.sent_off[0];
    // sentences of partition p
    int64_t lo = D.doc_sent_off[D.part_doc_off[p]], hi = D.doc_sent_off[D.part_doc_off[p + 1]] - 1;
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (D.sent_off[mid] <= x) lo = mid;
      else hi = mid - 1;
    }
    int64_t dlo = D.part_doc_off[p], dhi = D.part_doc_off[p + 1] - 1;
    while (dlo < dhi) {
      const int64_t mid = (dlo + dhi + 1) >> 1;
      if (D.doc_sent_off[mid] <= lo) dlo = mid;
      else dhi = mid - 1;
    }
    D.out_doc[g] = dlo;
  }
}

// np.save bytes of each row's masked positions (pretrain.py:356-360 stores
// serialize_np_array(np.array(positions, np.uint16)), lddl/utils.py:98-102)
__global__ __launch_bounds__(256) void npy_len_kernel(NpyParams N) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N.n_rows; i += stride) {
    int64_t k = N.moff[N.row0 + i + 1] - N.moff[N.row0 + i];
    if (k < 0 || k > N.kmax) {
      N.err[0] = 1;
      k = 0;
    }
    N.lens[i] = 2 * (N.hdr_u16 + (int32_t)k);
  }
}

// a wave per row, one u16 per lane (every row starts at an even byte offset)
__global__ __launch_bounds__(256) void npy_bytes_kernel(NpyParams N) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t o0 = N.out_off[0];
  for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < N.n_rows; i += nw) {
    const int64_t m0 = N.moff[N.row0 + i];
    const int32_t k = (int32_t)(N.moff[N.row0 + i + 1] - m0);
    uint16_t* dst = reinterpret_cast<uint16_t*>(N.out + (N.out_off[i] - o0));
    const uint16_t* h = N.hdr + (int64_t)k * N.hdr_u16;
    for (int32_t u = lane; u < N.hdr_u16 + k; u += 64) dst[u] = u < N.hdr_u16 ? h[u] : N.mpos[m0 + (u - N.hdr_u16)];
  }
}

static unsigned grid_for(int64_t waves, int n_cu) {
  const int64_t cap = (int64_t)n_cu * 32;  // 32 blocks (128 waves) per CU, grid-stride beyond
  int64_t b = (waves + 3) / 4;
  if (b > cap) b = cap;
  return (unsigned)(b < 1 ? 1 : b);
}

hipError_t launch_render_len(const RenderParams& R, int n_cu, hipStream_t s) {
  if (R.n_rows == 0) return hipSuccess;
  hipLaunchKernelGGL(render_len_kernel, dim3(grid_for(R.n_rows, n_cu)), dim3(256), 0, s, R);
  return hipGetLastError();
}

hipError_t launch_render_bytes(const RenderParams& R, int n_cu, hipStream_t s) {
  if (R.n_rows == 0) return hipSuccess;
  hipLaunchKernelGGL(render_bytes_kernel, dim3(grid_for(R.n_rows, n_cu)), dim3(256), 0, s, R);
  return hipGetLastError();
}

hipError_t launch_npy_len(const NpyParams& N, int n_cu, hipStream_t s) {
  if (N.n_rows == 0) return hipSuccess;
  int64_t b = (N.n_rows + 255) / 256, cap = (int64_t)n_cu * 16;
  hipLaunchKernelGGL(npy_len_kernel, dim3((unsigned)(b < cap ? b : cap)), dim3(256), 0, s, N);
  return hipGetLastError();
}

hipError_t launch_npy_bytes(const NpyParams& N, int n_cu, hipStream_t s) {
  if (N.n_rows == 0) return hipSuccess;
  hipLaunchKernelGGL(npy_bytes_kernel, dim3(grid_for(N.n_rows, n_cu)), dim3(256), 0, s, N);
  return hipGetLastError();
}

hipError_t launch_row_docs(const RowDocParams& D, int n_cu, hipStream_t s) {
  if (D.n_rows == 0) return hipSuccess;
  int64_t b = (D.n_rows + 255) / 256, cap = (int64_t)n_cu * 16;
  hipLaunchKernelGGL(row_docs_kernel, dim3((unsigned)(b < cap ? b : cap)), dim3(256), 0, s, D);
  return hipGetLastError();
}

}  // namespace lddl
