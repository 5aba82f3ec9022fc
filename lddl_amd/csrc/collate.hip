// Training-time collate: parquet rows -> BERT model inputs, and the dynamic
// 80/10/10 MLM masking, on the GPU.
//
// Reference: lddl/torch/bert.py:69-153 `_to_encoded_inputs` and :156-196
// `_mask_tokens`.  Per row: A.split() / B.split() (Python str.split: runs of
// Unicode whitespace), convert_tokens_to_ids (vocab lookup, [UNK] for a miss),
// tokens = [CLS] A [SEP] B [SEP] padded with 0 to the batch's longest row
// rounded up to `sequence_length_alignment`; token_type_ids 1 on B and its
// [SEP]; attention_mask 1 on the row; next_sentence_labels = is_random_next.
// Static masking (bert.py:113-116): labels = ignore_index except
// labels[positions] = ids(masked_lm_labels.split()), positions decoded from the
// row's np.save bytes.  Dynamic (bert.py:117-122, 156-196): special_tokens_mask
// = [CLS], the middle [SEP] and everything from the last [SEP] on; a
// non-special column is masked with probability mlm_probability, then [MASK]
// with p 0.8, else a random id in [0, len(tokenizer)) with p 0.5, else kept;
// labels = original id on masked columns, ignore_index elsewhere.  The draws
// come from a counter-based hash of (seed, counter, row, column) instead of
// torch's CPU generator: same distribution, not the same stream.
//
// Work mapping: one wave per row.  Pass 1 (token scan) walks the segment's
// bytes 64 at a time: lane i owns byte i, a token starts where a
// non-whitespace character follows whitespace; the token's ordinal is the
// ballot prefix count, the owning lane reads the token to its end, hashes it
// and probes the L2-resident vocab table.  Ids land in a per-wave LDS row;
// pass 2 writes the five int64 columns coalesced (lane = column).  The bound
// is the int64 output stream (40 B per column) against a few bytes of input.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "collate.h"
#include "wave.h"

namespace lddl {

static constexpr uint32_t kEmpty = 0xFFFFFFFFu;

__host__ __device__ __forceinline__ uint32_t chash_step(uint32_t h, uint32_t b) {
  h ^= b;
  return h * 0x01000193u;  // FNV-1a 32
}

__host__ __device__ __forceinline__ uint32_t chash_final(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7feb352du;
  h ^= h >> 15;
  h *= 0x846ca68bu;
  h ^= h >> 16;
  return h;
}

uint32_t collate_hash_host(const uint8_t* p, int n) {
  uint32_t h = 0x811c9dc5u;
  for (int i = 0; i < n; ++i) h = chash_step(h, p[i]);
  return chash_final(h);
}

// Python str.isspace() for the characters str.split() splits on
__device__ __forceinline__ bool py_space(uint32_t c) {
  if (c < 0x80) return (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x20);
  return c == 0x85 || c == 0xa0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200a) || c == 0x2028 || c == 0x2029 ||
         c == 0x202f || c == 0x205f || c == 0x3000;
}

// decode the UTF-8 character starting at p[i] (a lead byte), i < e
__device__ __forceinline__ uint32_t decode_at(const uint8_t* p, int64_t i, int64_t e, int& n) {
  const uint32_t b = p[i];
  if (b < 0x80) {
    n = 1;
    return b;
  }
  n = b >= 0xF0 ? 4 : b >= 0xE0 ? 3 : 2;
  uint32_t c = b & (0x7Fu >> n);
  for (int k = 1; k < n; ++k) c = (c << 6) | (i + k < e ? (p[i + k] & 0x3Fu) : 0u);
  return c;
}

// does byte i (s <= i < e) belong to a whitespace character?
__device__ __forceinline__ bool ws_byte(const uint8_t* p, int64_t i, int64_t s, int64_t e) {
  const uint32_t b = p[i];
  if (b < 0x80) return py_space(b);
  int64_t j = i;
  while (j > s && j > i - 3 && (p[j] & 0xC0u) == 0x80u) --j;
  int n;
  return py_space(decode_at(p, j, e, n));
}

__device__ __forceinline__ int32_t vocab_lookup(const CollateVocab& V, const uint8_t* p, int64_t i, int64_t e,
                                                int64_t& end) {
  uint32_t h = 0x811c9dc5u;
  int64_t j = i;
  while (j < e) {
    const uint32_t b = p[j];
    if (b < 0x80) {
      if (py_space(b)) break;
      h = chash_step(h, b);
      ++j;
      continue;
    }
    int n;
    const uint32_t c = decode_at(p, j, e, n);
    if (py_space(c)) break;
    for (int k = 0; k < n && j + k < e; ++k) h = chash_step(h, p[j + k]);
    j += n;
  }
  if (j > e) j = e;
  end = j;
  h = chash_final(h);
  const uint32_t len = (uint32_t)(j - i);
  for (uint32_t s = h & V.mask;; s = (s + 1) & V.mask) {
    const uint2 t = V.slots[s];
    if (t.y == kEmpty) return V.unk;
    if (t.x != h) continue;
    const uint32_t vi = V.vinfo[t.y];
    if ((vi & 0xFFu) != len) continue;
    const uint8_t* q = V.vpool + (vi >> 8);
    uint32_t k = 0;
    while (k < len && q[k] == p[i + k]) ++k;
    if (k == len) return (int32_t)t.y;
  }
}

// Walk the tokens of bytes [s, e): calls f(ordinal, start) on the owning lane
// (ordinal in token order); returns the token count (wave-uniform).
template <class F>
__device__ __forceinline__ int32_t scan_tokens(const uint8_t* p, int64_t s, int64_t e, F f) {
  const int lane = threadIdx.x & 63;
  int32_t count = 0;
  for (int64_t base = s; base < e; base += 64) {
    const int64_t i = base + lane;
    bool st = false;
    if (i < e) {
      const uint32_t b = p[i];
      st = (b & 0xC0u) != 0x80u && !ws_byte(p, i, s, e) && (i == s || ws_byte(p, i - 1, s, e));
    }
    const uint64_t m = __ballot(st);
    if (st) f(count + (int32_t)__popcll(m & ((1ull << lane) - 1ull)), i);
    count += (int32_t)__popcll(m);
  }
  return count;
}

__device__ __forceinline__ void set_err(uint32_t* err, uint32_t code, int64_t row) {
  atomicCAS(err, 0u, code | ((uint32_t)row << 4));
}

// max_len = max over rows of len(A) + len(B) + 3
__global__ __launch_bounds__(256) void collate_len_kernel(CollateParams P) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < P.n_rows; r += nw) {
    auto none = [](int32_t, int64_t) {};
    const int32_t na = scan_tokens(P.a, P.a_off[r], P.a_off[r + 1], none);
    const int32_t nb = scan_tokens(P.b, P.b_off[r], P.b_off[r + 1], none);
    if (lane == 0) atomicMax(P.max_len, na + nb + 3);
  }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ double unit53(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }

// _mask_tokens for one column: returns the (possibly replaced) input id and
// sets label
__device__ __forceinline__ int64_t mask_one(int64_t id, bool special, int64_t row, int32_t col, uint64_t seed,
                                            uint64_t counter, double p, int32_t mask_id, int32_t n_random,
                                            int64_t ignore, int64_t& label) {
  const uint64_t k = splitmix64(seed ^ splitmix64(counter));
  const uint64_t idx = ((uint64_t)row << 20 | (uint64_t)col) * 3ull;
  label = ignore;
  if (special || !(unit53(splitmix64(k + idx)) < p)) return id;
  label = id;
  const uint64_t h = splitmix64(k + idx + 1);
  if (unit53(h) < 0.8) return mask_id;
  const uint64_t g = splitmix64(k + idx + 2);
  if (unit53(g) < 0.5) return (int64_t)(((g & 0xFFFFFFFFull) * (uint64_t)n_random) >> 32);
  return id;
}

__global__ __launch_bounds__(256) void collate_fill_kernel(CollateParams P) {
  __shared__ int32_t s_ids[4][COLLATE_MAX_LEN];
  __shared__ int32_t s_lab[4][COLLATE_MAX_LEN];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  int32_t* ids = s_ids[w];
  int32_t* lab = s_lab[w];
  const int32_t L = P.seq_len;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + w; r < P.n_rows; r += nw) {
    const CollateVocab& V = P.V;
    // pass 1: token ids into the LDS row (positions >= L are dropped and flagged)
    int32_t na = scan_tokens(P.a, P.a_off[r], P.a_off[r + 1], [&](int32_t k, int64_t i) {
      int64_t end;
      const int32_t id = vocab_lookup(V, P.a, i, P.a_off[r + 1], end);
      if (1 + k < L) ids[1 + k] = id;
    });
    int32_t nb = scan_tokens(P.b, P.b_off[r], P.b_off[r + 1], [&](int32_t k, int64_t i) {
      int64_t end;
      const int32_t id = vocab_lookup(V, P.b, i, P.b_off[r + 1], end);
      if (na + 2 + k < L) ids[na + 2 + k] = id;
    });
    const int32_t n = na + nb + 3;
    if (n > L) {
      if (lane == 0) set_err(P.err, CERR_LONG, r);
      continue;
    }
    if (P.mode == COLLATE_STATIC) {
      for (int32_t j = lane; j < L; j += 64) lab[j] = -1;
      // positions: np.save v1.x bytes of a 1-D '<u2' array
      const uint8_t* q = P.pos + P.pos_off[r];
      const int64_t qn = P.pos_off[r + 1] - P.pos_off[r];
      bool ok = qn >= 10 && q[0] == 0x93 && q[1] == 'N' && q[2] == 'U' && q[3] == 'M' && q[4] == 'P' &&
                q[5] == 'Y' && q[6] == 1;
      const int64_t hl = ok ? (int64_t)q[8] | ((int64_t)q[9] << 8) : 0;
      ok = ok && 10 + hl <= qn && ((qn - 10 - hl) & 1) == 0;
      if (!ok) {
        if (lane == 0) set_err(P.err, CERR_NPY, r);
        continue;
      }
      const int32_t np = (int32_t)((qn - 10 - hl) >> 1);
      const uint8_t* d = q + 10 + hl;
      __builtin_amdgcn_wave_barrier();
      // labels[positions[k]] = id(masked_lm_labels.split()[k])
      const int64_t l0 = P.lab_off[r], l1 = P.lab_off[r + 1];
      bool bad = false;
      const int32_t nl = scan_tokens(P.lab, l0, l1, [&](int32_t k, int64_t i) {
        int64_t end;
        const int32_t id = vocab_lookup(V, P.lab, i, l1, end);
        if (k < np) {
          const int32_t pos = (int32_t)d[2 * k] | ((int32_t)d[2 * k + 1] << 8);
          if (pos >= L) bad = true;
          else lab[pos] = id;
        }
      });
      if (nl != np) {
        if (lane == 0) set_err(P.err, CERR_NLAB, r);
        continue;
      }
      if (__ballot(bad)) {
        if (lane == 0) set_err(P.err, CERR_POS_RANGE, r);
        continue;
      }
    }
    __builtin_amdgcn_wave_barrier();
    // pass 2: the int64 columns, lane = column
    int64_t* o_ids = P.input_ids + r * (int64_t)L;
    int64_t* o_tt = P.token_type_ids + r * (int64_t)L;
    int64_t* o_am = P.attention_mask + r * (int64_t)L;
    int64_t* o_lab = P.labels + r * (int64_t)L;
    for (int32_t j = lane; j < L; j += 64) {
      int64_t id;
      if (j == 0) id = V.cls;
      else if (j == na + 1 || j == n - 1) id = V.sep;
      else if (j < n) id = ids[j];
      else id = 0;
      const bool special = j == 0 || j == na + 1 || j >= n - 1;
      int64_t l;
      if (P.mode == COLLATE_SPECIAL_MASK) l = special ? 1 : 0;
      else if (P.mode == COLLATE_STATIC) l = lab[j] < 0 ? P.ignore_index : (int64_t)lab[j];
      else id = mask_one(id, special, r, j, P.seed, P.counter, P.mlm_probability, V.mask_id, V.n_random,
                         P.ignore_index, l);
      o_ids[j] = id;
      o_tt[j] = (j >= na + 2 && j < n) ? 1 : 0;
      o_am[j] = j < n ? 1 : 0;
      o_lab[j] = l;
    }
    if (lane == 0) P.next_sentence_labels[r] = P.is_random_next[r] ? 1 : 0;
  }
}

__global__ __launch_bounds__(256) void mask_tokens_kernel(MaskParams M) {
  const int64_t total = M.n_rows * (int64_t)M.seq_len;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t r = e / M.seq_len;
    const int32_t j = (int32_t)(e - r * M.seq_len);
    int64_t l;
    M.inputs[e] = mask_one(M.inputs[e], M.special[e] != 0, r, j, M.seed, M.counter, M.mlm_probability, M.mask_id,
                           M.n_random, M.ignore_index, l);
    M.labels[e] = l;
  }
}

static int grid_rows(int64_t n_rows, int n_cu) {
  int64_t g = (n_rows + 3) / 4;
  const int64_t cap = (int64_t)n_cu * 8;
  if (g > cap) g = cap;
  return (int)(g < 1 ? 1 : g);
}

hipError_t launch_collate_len(const CollateParams& P, int n_cu, hipStream_t s) {
  if (P.n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(collate_len_kernel, dim3(grid_rows(P.n_rows, n_cu)), dim3(256), 0, s, P);
  return hipGetLastError();
}

hipError_t launch_collate_fill(const CollateParams& P, int n_cu, hipStream_t s) {
  if (P.n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(collate_fill_kernel, dim3(grid_rows(P.n_rows, n_cu)), dim3(256), 0, s, P);
  return hipGetLastError();
}

hipError_t launch_mask_tokens(const MaskParams& M, int n_cu, hipStream_t s) {
  const int64_t total = M.n_rows * (int64_t)M.seq_len;
  if (total <= 0) return hipSuccess;
  int64_t g = (total + 255) / 256;
  if (g > (int64_t)n_cu * 16) g = (int64_t)n_cu * 16;
  hipLaunchKernelGGL(mask_tokens_kernel, dim3((int)g), dim3(256), 0, s, M);
  return hipGetLastError();
}

}  // namespace lddl
