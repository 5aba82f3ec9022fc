// Tile bounds and the exact serial tokenizer path.
//
// Tiles: tile t owns the sentences whose first byte lies in
// [t * 1 KiB, (t+1) * 1 KiB) (relative to sent_off[0]); no sentence crosses a
// tile, so every tile is independent.  tile_sent[t] = first sentence of tile
// t (tile_bounds_kernel, one pass over the sentences).
//
// tokenize_fallback_kernel re-runs listed sentence ranges (the split
// tokenizer's scan windows it did not model, or whole tiles) one lane per sentence
// (tokenize_serial.h: the serial restatement of HF tokenizers'
// BertNormalizer / BertPreTokenizer / WordPiece behind
// tokenizer.tokenize(s, max_length=512, truncation=True),
// lddl/dask/bert/pretrain.py:79-80, as oracle/tokenizer_oracle.c).  The
// split tokenizer (tokenize_split.hip) lists the windows it does not model;
// launch_tokenize_serial_dense lists every tile (vocabularies / unicode
// tables the split tokenizer does not take: > 61440 ids, or an ASCII page
// with more than the A-Z -> a-z mapping).  Its ids are written sparse by
// byte offset (P.out_ids + sent_off[s] - sent_off[0]) into the split path's
// entry buffer, from which expand_kernel writes the dense output.
#include <algorithm>

#include "common.h"
#include "tokenize.h"
#include "tokenize_serial.h"

namespace lddl {

constexpr int TILE_SHIFT = 10;  // nominal tile: sentences starting in 1 KiB

// tile_sent[t] = first sentence whose start (relative) >= t * TILE, for the
// tiles t the caller reads: (t % seg) % sup == 0 (the split scan's
// super-tile starts in each segment of seg tiles; sup = 1: every tile) and
// t = n_tiles
__global__ void tile_bounds_kernel(const int64_t* sent_off, int64_t n_sent, int64_t n_tiles, int64_t* tile_sent,
                                   int64_t* tile_off, int64_t seg, int sup) {
  const int64_t base = sent_off[0];
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= n_sent; s += (int64_t)gridDim.x * blockDim.x) {
    // tiles t with off[s-1] < t*TILE <= off[s] map to s (s = n_sent: the rest)
    const int64_t hi = s < n_sent ? sent_off[s] - base : (n_tiles << TILE_SHIFT);
    const int64_t lo = s > 0 ? sent_off[s - 1] - base : -1;
    int64_t t0 = (lo >> TILE_SHIFT) + 1;  // first t with t*TILE > lo
    if (lo < 0) t0 = 0;
    const int64_t t1 = hi >> TILE_SHIFT;  // last t with t*TILE <= hi
    for (int64_t t = t0; t <= t1 && t <= n_tiles; ++t) {
      if ((t % seg) % sup != 0 && t != n_tiles) continue;
      tile_sent[t] = s;
      if (tile_off) tile_off[t] = sent_off[s];
    }
  }
}

// The same bounds for the super-tile starts alone (sup > 1): a lower-bound
// search per tile read (first s with sent_off[s] - base >= t * TILE; n_sent if
// none) instead of a pass over every sentence offset -- ~1/16 of the tiles
__global__ void tile_bounds_search_kernel(const int64_t* sent_off, int64_t n_sent, int64_t n_tiles, int64_t* tile_sent,
                                          int64_t* tile_off, int64_t seg, int sup) {
  const int64_t base = sent_off[0];
  const int64_t per_seg = (seg + sup - 1) / sup, nseg = n_tiles > 0 ? (n_tiles + seg - 1) / seg : 0;
  const int64_t core = nseg > 0 ? (nseg - 1) * per_seg + (n_tiles - (nseg - 1) * seg + sup - 1) / sup : 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= core; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i == core ? n_tiles : (i / per_seg) * seg + (i % per_seg) * sup;  // (i == core: the end)
    const int64_t x = t << TILE_SHIFT;
    int64_t lo = 0, hi = n_sent;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (sent_off[mid] - base < x) lo = mid + 1;
      else hi = mid;
    }
    tile_sent[t] = lo;
    if (tile_off) tile_off[t] = sent_off[lo];
  }
}

// Exact serial path for the listed sentence ranges (a scan window or a tile
// the split tokenizer did not model): lane per sentence (tokenize_serial.h).
__global__ __launch_bounds__(256) void tokenize_fallback_kernel(TokParams P, const int64_t* fb_list,
                                                                const int32_t* fb_count) {
  __shared__ uint32_t ascii_tab[128];
  if (threadIdx.x < 128) ascii_tab[threadIdx.x] = P.pages[(uint32_t)P.top[0] * 256u + threadIdx.x];
  __syncthreads();
  const int n = *fb_count;
  const LdsWordBuf wb{P.ovf + ((size_t)blockIdx.x * 256 + threadIdx.x) * WB_OVF};
  const int64_t base = P.sent_off[0];
  const int wave = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const int nw = (gridDim.x * 256) >> 6;
  for (int k = wave; k < n; k += nw) {
    const int64_t sa = fb_list[2 * k], sb = fb_list[2 * k + 1];
    for (int64_t s = sa + lane; s < sb; s += 64) {
      SentState st{P.sent_off[s], P.sent_off[s + 1], P.sent_off[s] - base, 0};
      while (st.p < st.e && st.ntok < P.max_tok) step(P, st, wb, ascii_tab);
      const int nt = min(st.ntok, P.max_tok);
      P.out_ntok[s] = nt;
      if (P.sent_spec) {  // the sentence holds a [CLS] / [SEP] token
        const uint16_t* ids = P.out_ids + (P.sent_off[s] - base);
        uint32_t f = 0;
        for (int k = 0; k < nt; ++k) f |= (ids[k] == P.special[2]) | (ids[k] == P.special[3]);
        P.sent_spec[s] = (uint8_t)f;
      }
    }
  }
}

int64_t tile_count(int64_t nbytes) { return (nbytes >> TILE_SHIFT) + 1; }
// (the scan's windows: two consecutive windows of a super-tile cover more
// than 2 KiB - 16 B, a window longer than 2 KiB holds one sentence, plus a
// partly filled last window per super-tile -> fewer than 2 per tile; the
// serial path lists one range per tile)
int64_t fb_list_cap(int64_t seg_tiles) { return 2 * (2 * seg_tiles + 64); }
const void* tokenize_fallback_kernel_ptr() { return reinterpret_cast<const void*>(&tokenize_fallback_kernel); }


__global__ void list_all_tiles_kernel(int64_t n_tiles, const int64_t* tile_sent, int64_t* fb_list,
                                      int32_t* fb_count) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_tiles; t += (int64_t)gridDim.x * blockDim.x) {
    fb_list[2 * t] = tile_sent[t];
    fb_list[2 * t + 1] = tile_sent[t + 1];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *fb_count = (int32_t)n_tiles;
}

hipError_t launch_list_all_tiles(int64_t n_tiles, const int64_t* tile_sent, int64_t* fb_list, int32_t* fb_count,
                                 hipStream_t s) {
  hipLaunchKernelGGL(list_all_tiles_kernel, dim3(1024), dim3(256), 0, s, n_tiles, tile_sent, fb_list, fb_count);
  return hipGetLastError();
}

hipError_t launch_tile_bounds(const int64_t* sent_off, int64_t n_sent, int64_t n_tiles, int64_t* tile_sent,
                              int64_t* tile_off, hipStream_t s, int64_t seg, int sup) {
  const int64_t sg = seg > 0 ? seg : n_tiles + 1;
  if (sup > 1) {
    const int64_t need = n_tiles / sup + (n_tiles + sg - 1) / sg + 1;  // (>= the tiles searched)
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((need + 255) / 256, 4096));
    hipLaunchKernelGGL(tile_bounds_search_kernel, dim3(grid), dim3(256), 0, s, sent_off, n_sent, n_tiles, tile_sent,
                       tile_off, sg, sup);
  } else {
    hipLaunchKernelGGL(tile_bounds_kernel, dim3(4096), dim3(256), 0, s, sent_off, n_sent, n_tiles, tile_sent, tile_off,
                       sg, 1);
  }
  return hipGetLastError();
}

hipError_t launch_tokenize_fallback(const TokParams& P, const int64_t* fb_list, const int32_t* fb_count, int grid,
                                    hipStream_t s) {
  hipLaunchKernelGGL(tokenize_fallback_kernel, dim3(grid), dim3(256), 0, s, P, fb_list, fb_count);
  return hipGetLastError();
}

}  // namespace lddl
