// Standalone sequence-length binning (lddl_bin): the grouping of
// lddl/dask/bert/binning.py:63-93 _to_dataframe_binned over any column of
// row lengths, as a stable counting sort by bin.
//
//   bin(len) = (len - 1) // bin_size   (Python floor division)
//              -> nbins - 1 when above it; a negative bin indexes the bin
//              list from the end as Python's seqs[bin_id] does (len 0 ->
//              the last bin), below -nbins the reference's IndexError
//
// A wave owns a chunk of BIN_CHUNK rows and walks it 64 rows at a time in row
// order: the lanes holding the same bin find each other with one ballot per
// bit of the bin id, a lane's rank among them is a popcount below it, and the
// lowest such lane adds the group's size to the chunk's per-bin counter in
// LDS (the group leaders hold distinct bins: no atomics).  Pass 1 writes the
// chunk's counters bin-major (hist[bin][chunk]); an exclusive scan of that
// array is every (bin, chunk)'s first output row; pass 2 walks the chunk again
// and scatters row indices.  HBM-bound: 8 B read per row per pass, 8 B written.
#include "pack.h"
#include "wave.h"

namespace lddl {

namespace {

constexpr int BIN_CHUNK = 4096;  // rows per wave
constexpr int BIN_WAVES = 4;     // waves per workgroup
constexpr int BIN_UNROLL = 16;   // 64-row groups loaded ahead

__device__ __forceinline__ int32_t bin_of(int64_t len, int32_t bin_size, int32_t nbins) {
  const int64_t x = len - 1;
  int64_t b = x >= 0 ? x / bin_size : -((-x + bin_size - 1) / bin_size);
  if (b > nbins - 1) b = nbins - 1;
  if (b < 0) b += nbins;
  return b < 0 ? -1 : (int32_t)b;
}

// lanes of the wave holding the same value v (nbits low bits) among `act`
__device__ __forceinline__ uint64_t peers(uint32_t v, int nbits, uint64_t act) {
  uint64_t m = act;
  for (int k = 0; k < nbits; ++k) {
    const uint64_t b = __ballot((v >> k) & 1);
    m &= ((v >> k) & 1) ? b : ~b;
  }
  return m;
}

template <bool SCATTER>
__global__ __launch_bounds__(64 * BIN_WAVES) void bin_kernel(const int64_t* __restrict__ num_tokens, int64_t n,
                                                            int32_t bin_size, int32_t nbins, int nbits,
                                                            int64_t nchunks, int32_t* __restrict__ hist,
                                                            const int64_t* __restrict__ base,
                                                            int64_t* __restrict__ perm, int32_t* __restrict__ err,
                                                            int64_t* __restrict__ bin_counts) {
  extern __shared__ int64_t run_lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int64_t* run = run_lds + (size_t)w * nbins;
  const int64_t chunk = (int64_t)blockIdx.x * BIN_WAVES + w;
  if (SCATTER && chunk == 0)
    for (int b = lane; b < nbins; b += 64) bin_counts[b] = base[(int64_t)(b + 1) * nchunks] - base[(int64_t)b * nchunks];
  if (chunk >= nchunks) return;
  for (int b = lane; b < nbins; b += 64) run[b] = SCATTER ? base[(int64_t)b * nchunks + chunk] : 0;
  const int64_t r0 = chunk * BIN_CHUNK;
  const int64_t r1 = r0 + BIN_CHUNK < n ? r0 + BIN_CHUNK : n;
  for (int64_t g = r0; g < r1; g += 64 * BIN_UNROLL) {
    int64_t v[BIN_UNROLL];
#pragma unroll
    for (int u = 0; u < BIN_UNROLL; ++u) {
      const int64_t i = g + u * 64 + lane;
      v[u] = i < r1 ? num_tokens[i] : 1;
    }
#pragma unroll
    for (int u = 0; u < BIN_UNROLL; ++u) {
      const int64_t i = g + u * 64 + lane;
      if (g + u * 64 >= r1) break;  // wave-uniform
      const bool in = i < r1;
      int32_t b = bin_of(v[u], bin_size, nbins);
      if (in && b < 0) {
        if (!SCATTER) err[0] = 1;
        b = 0;
      }
      const uint64_t m = peers((uint32_t)b, nbits, __ballot(in));
      const int rank = bits_below(m);
      const int64_t at = run[b];
      if (SCATTER && in) perm[at + rank] = i;
      if (in && rank == 0) run[b] = at + __builtin_popcountll(m);
    }
  }
  if (!SCATTER)
    for (int b = lane; b < nbins; b += 64) hist[(int64_t)b * nchunks + chunk] = (int32_t)run[b];
}

}  // namespace

int64_t bin_chunks(int64_t n) { return (n + BIN_CHUNK - 1) / BIN_CHUNK; }

hipError_t launch_bin(const int64_t* num_tokens, int64_t n, int32_t bin_size, int32_t nbins, int32_t* hist,
                      int64_t* base, int64_t* scan_bsum, int64_t* perm, int64_t* bin_counts, int32_t* err,
                      hipStream_t s) {
  const int64_t nchunks = bin_chunks(n);
  int nbits = 0;
  while ((1 << nbits) < nbins) ++nbits;
  const size_t lds = (size_t)BIN_WAVES * nbins * sizeof(int64_t);
  const dim3 grid((unsigned)((nchunks + BIN_WAVES - 1) / BIN_WAVES));
  hipError_t e;
  if ((e = hipMemsetAsync(err, 0, sizeof(int32_t), s))) return e;
  if (nchunks == 0) return hipMemsetAsync(bin_counts, 0, (size_t)nbins * sizeof(int64_t), s);
  hipLaunchKernelGGL(bin_kernel<false>, grid, dim3(64 * BIN_WAVES), lds, s, num_tokens, n, bin_size, nbins, nbits,
                     nchunks, hist, (const int64_t*)nullptr, (int64_t*)nullptr, err, (int64_t*)nullptr);
  if ((e = hipGetLastError())) return e;
  if ((e = launch_scan_ntok(hist, nchunks * nbins, base, scan_bsum, s))) return e;
  hipLaunchKernelGGL(bin_kernel<true>, grid, dim3(64 * BIN_WAVES), lds, s, num_tokens, n, bin_size, nbins, nbits,
                     nchunks, (int32_t*)nullptr, (const int64_t*)base, perm, err, bin_counts);
  return hipGetLastError();
}

}  // namespace lddl
