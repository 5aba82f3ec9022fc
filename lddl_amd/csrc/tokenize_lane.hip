// Lane tokenizer (tok6, default): tokenize_lane.h's per-lane walk as a
// persistent wave of 64 lanes, then the dense CSR output.
//
// Contract: lddl_tokenize (include/lddl_amd.h) = HF tokenizers behind
// tokenizer.tokenize(s, max_length=512, truncation=True),
// lddl/dask/bert/pretrain.py:79-80 (oracle/tokenizer_oracle.c).
//
// Per segment of tiles (SPLIT_SEG_TILES):
//   lane_kernel     waves take batches of LANE_BATCH tiles from a counter;
//                   a lane takes the batch's next tile whenever it finishes
//                   one (so lanes stay busy until the segment's last batch).
//                   Each lane's bytes stream into its own 64-B ring in LDS by
//                   LDS-DMA, every REFILL_EVERY iterations for all lanes at
//                   once (one HBM round trip per 16 iterations instead of one
//                   per lane crossing); per iteration every lane consumes one
//                   byte (tokenize_lane.h).  Ids are staged at the sentence's
//                   byte offset (u16 per input byte), counts go to out_ntok.
//   fallback        the exact serial path over tiles a lane gave up on (a
//                   normalised word longer than the ring)
//   scan            out_ntok -> out_tok_off (continuing the last segment)
//   compact_kernel  staged ids -> the dense output, a wave per 64 sentences,
//                   one token per lane per step
#include "common.h"
#include "tokenize.h"
#include "tokenize_lane.h"
#include "wave.h"
#include "pack.h"

namespace lddl {
namespace tok6 {

constexpr int LWAVES = 4;  // waves per workgroup

struct DevEnv {
  const TokParams& P;
  const LaneParams& Q;
  uint8_t* ring;            // this lane's 16 B of ring slot 0; slot k 1 KiB further (LDS)
  const uint16_t* ct;       // byte classes (LDS)
  const uint32_t* asct;     // unicode entries of the ASCII page (LDS)
  __device__ __forceinline__ uint32_t rbyte(int32_t q) const {
    return ring[((q >> 4) & (RING_SLOTS - 1)) * 1024 + (q & 15)];
  }
  __device__ __forceinline__ uint32_t ctab(uint32_t b) const { return ct[b]; }
  __device__ __forceinline__ uint2 trie(uint32_t i) const { return Q.trie[i]; }
  __device__ __forceinline__ uint32_t bget(int i) const { return rbyte(i); }
  __device__ __forceinline__ void bput(int i, uint32_t v) const {
    // (dword read-modify-write: byte-typed LDS stores trip a gfx950 isel bug, tokenize_serial.h)
    uint32_t* w = reinterpret_cast<uint32_t*>(ring + ((i >> 4) & (RING_SLOTS - 1)) * 1024 + (i & 12));
    const int sh = (i & 3) * 8;
    *w = (*w & ~(0xFFu << sh)) | ((v & 0xFFu) << sh);
  }
  __device__ __forceinline__ uint32_t raw(int64_t a) const { return P.bytes[a]; }
  __device__ __forceinline__ uint32_t asc(uint32_t b) const { return asct[b]; }
  __device__ __forceinline__ void put_tok(int64_t i, uint32_t id) const { Q.stage[i] = (uint16_t)id; }
  __device__ __forceinline__ int64_t soff(int64_t i) const { return P.sent_off[i]; }
  __device__ __forceinline__ void put_ntok(int64_t s, int32_t n, uint32_t spec) const {
    P.out_ntok[s] = n;
    if (P.sent_spec) P.sent_spec[s] = (uint8_t)spec;
  }
  __device__ __forceinline__ void abort_tile(const LaneState& L) const {
    const int at = atomicAdd(Q.fb_count, 1);
    Q.fb_list[2 * at] = Q.tile_sent[L.t];
    Q.fb_list[2 * at + 1] = Q.tile_sent[L.t + 1];
    atomicAdd(Q.n_fallback, 1u);
  }
};

// DBG: phase stamps (s_memtime, wave-summed) into Q.stats[3..]: hand-out,
// refill (with its wait), slow pass, step
template <int WAVES, bool DBG>
__global__ __launch_bounds__(64 * WAVES) void lane_kernel(TokParams P, LaneParams Q0, const uint16_t* g_ctab) {
  uint64_t acc[4] = {0, 0, 0, 0}, tprev = 0;
#define LSTAMP(k)                                                                \
  if (DBG) {                                                                     \
    uint64_t t_;                                                                 \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    acc[k] += t_ - tprev;                                                        \
    tprev = t_;                                                                  \
  }
  LaneParams Q = Q0;
  Q.segb += P.sent_off[0];  // (staging index 0 = the segment's first byte)
  Q.bytes_end = P.sent_off[P.n_sent];
  __shared__ __attribute__((aligned(16))) uint8_t rings[WAVES][RING_SLOTS][1024];
  __shared__ uint16_t ct[256];
  __shared__ uint32_t asct[128];
  for (int i = threadIdx.x; i < 256; i += 64 * WAVES) ct[i] = g_ctab[i];
  for (int i = threadIdx.x; i < 128; i += 64 * WAVES) asct[i] = P.pages[(uint32_t)P.top[0] * 256u + i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const DevEnv en{P, Q, &rings[wv][0][0] + lane * 16, ct, asct};
  LaneState L{};
  L.mode = M_NEED;
  // the wave's batch of tiles [bnext, bend); lane 0 holds the next batch's
  // index, fetched one batch ahead so the atomic's round trip is hidden
  int64_t bnext = 0, bend = 0;
  bool exhausted = false;
  uint32_t nbat = 0;
  if (lane == 0) nbat = atomicAdd(Q.ctr, 1u);
  uint32_t iter = 0, slow_age = 0;
  uint64_t n_busy = 0, n_slow = 0;
  if (DBG) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tprev)::"memory");
  for (;;) {
    // ---- ring refill: every lane's missing 16-B chunks, all loads first, then
    //      their LDS stores (no LDS-DMA: LLVM would then put a vmcnt(0) wait
    //      in front of every ring read, serialising each iteration behind the
    //      previous one's stores); one HBM round trip per REFILL_EVERY
    //      iterations (vmcnt counts in order, so any later wait pays it anyway)
    if ((iter & (REFILL_EVERY - 1)) == 0) {
      const bool act = L.mode == M_SCAN || L.mode == M_WORD || L.mode == M_SKIP;
      int nload = 0;
      if (act) {
        const int32_t keep = (L.mode == M_WORD && L.la >= 0) ? L.la : L.p;
        if ((keep >> 4) > L.rlo) L.rlo = keep >> 4;
        if (L.rhi < L.rlo) L.rhi = L.rlo;
        const int64_t room = (Q.bytes_end - L.tb16 + 15) / 16 - L.rhi;  // chunks left before the corpus end
        nload = (int)min((int64_t)(L.rlo + RING_SLOTS - L.rhi), max(room, (int64_t)0));
      }
      // (RING_SLOTS loads per lane, every one issued before the first LDS
      // store -- a load per needed chunk under its own branch came out as
      // load, wait, store, load ...; lanes needing fewer re-load their last)
      if (__ballot(nload > 0)) {
        uint4 v[RING_SLOTS];
        const int64_t c0 = nload > 0 ? L.tb16 + 16 * (int64_t)L.rhi : 0;
#pragma unroll
        for (int r = 0; r < RING_SLOTS; ++r)
          v[r] = *reinterpret_cast<const uint4*>(P.bytes + c0 + 16 * (int64_t)min(r, max(nload - 1, 0)));
#pragma unroll
        for (int r = 0; r < RING_SLOTS; ++r)  // (keeps the loads from sinking into the stores' branches)
          asm volatile("" : "+v"(v[r].x), "+v"(v[r].y), "+v"(v[r].z), "+v"(v[r].w));
#pragma unroll
        for (int r = 0; r < RING_SLOTS; ++r)
          if (r < nload) *reinterpret_cast<uint4*>(&rings[wv][(L.rhi + r) & (RING_SLOTS - 1)][lane * 16]) = v[r];
      }
      L.rhi += nload;
    }
    LSTAMP(1)
    // ---- the batched slow path
    const uint64_t sw = __ballot(L.mode == M_SLOW);
    if (sw) {
      ++slow_age;
      const uint64_t other = __ballot(L.mode >= M_TILE && L.mode != M_SLOW);
      if (__popcll(sw) >= SLOW_BATCH || slow_age >= SLOW_AGE || other == 0) {
        if (L.mode == M_SLOW) lane_slow(L, en);
        slow_age = 0;
        ++n_slow;
      }
    }
    LSTAMP(2)
    if (Q.stats) n_busy += __popcll(__ballot(L.mode >= M_TILE && L.mode != M_SLOW));
    lane_step(L, en);
    if (DBG) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    LSTAMP(3)
    // ---- tiles for lanes that finished theirs, last in the iteration: the
    //      loads land during the next one's ring reads, where M_TILE reads them
    //      (issued earlier, their results would be waited for -- and, vmcnt
    //      counting in order, every store of the iteration with them)
    const uint64_t need = __ballot(L.mode == M_NEED);
    if (need) {
      if (bnext >= bend && !exhausted) {
        const int64_t b = Q.t0 + (int64_t)lane_get(nbat, 0) * LANE_BATCH;
        if (b < Q.t1) {
          bnext = b;
          bend = min(b + (int64_t)LANE_BATCH, Q.t1);
          if (lane == 0) nbat = atomicAdd(Q.ctr, 1u);
        } else {
          exhausted = true;
        }
      }
      if (L.mode == M_NEED) {
        const int64_t t = bnext + bits_below(need);
        if (t < bend) {
          L.t = t;
          L.s = Q.tile_sent[t];
          L.sb = Q.tile_sent[t + 1];
          L.obase = Q.tile_off[t];
          L.mode = M_TILE;
        } else if (exhausted) {
          L.mode = M_IDLE;
        }
      }
      bnext = min(bnext + (int64_t)__popcll(need), bend);
    }
    LSTAMP(0)
    ++iter;
    if (__ballot(L.mode != M_IDLE) == 0) break;
  }
  if (Q.stats && lane == 0) {
    atomicAdd((unsigned long long*)&Q.stats[0], (unsigned long long)iter * 64ull);
    atomicAdd((unsigned long long*)&Q.stats[1], (unsigned long long)n_busy);
    atomicAdd((unsigned long long*)&Q.stats[2], (unsigned long long)n_slow);
    if (DBG)
      for (int k = 0; k < 4; ++k) atomicAdd((unsigned long long*)&Q.stats[3 + k], (unsigned long long)acc[k]);
  }
#undef LSTAMP
}

// ------------------------------------------------------------- compact --
// staged ids (sentence s's at sent_off[s] - segb) -> out_ids[out_tok_off[s] ..]
// (capped at out_cap); a wave per 64 sentences, one token per lane per step,
// a token's sentence from a scatter of the sentences' first tokens + a wave
// max-scan (the packed output of consecutive sentences is contiguous, so a
// step's stores are one run)
__global__ __launch_bounds__(256) void compact_kernel(TokParams P, const uint16_t* stage, int64_t seg_rel,
                                                      const int64_t* tile_sent, int64_t t0, int64_t t1) {
  const int64_t segb = P.sent_off[0] + seg_rel;
  __shared__ uint32_t own_s[4][64];
  __shared__ int64_t src_s[4][64], dst_s[4][64];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* own = own_s[wv];
  const int64_t sA = tile_sent[t0], sB = tile_sent[t1];
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t g0 = sA + ((int64_t)blockIdx.x * 4 + wv) * 64; g0 < sB; g0 += nwaves * 64) {
    const int64_t s = g0 + lane;
    uint32_t n = 0;
    int64_t src = 0, dst = 0;
    if (s < sB) {
      dst = P.out_tok_off[s];
      const int64_t room = P.out_cap - dst;
      n = (uint32_t)max((int64_t)0, min((int64_t)P.out_ntok[s], room));
      src = P.sent_off[s] - segb;
    }
    const uint32_t x = wave_incl_add(n);
    const uint32_t e0 = x - n, T = lane_get(x, 63);
    src_s[wv][lane] = src - e0;
    dst_s[wv][lane] = dst - e0;
    uint32_t carry = 0;
    for (uint32_t st = 0; st < T; st += 64) {
      own[lane] = 0u;
      __builtin_amdgcn_wave_barrier();
      if (n != 0 && e0 >= st && e0 < st + 64) atomicMax(&own[e0 - st], (uint32_t)lane);
      __builtin_amdgcn_wave_barrier();
      const uint32_t o = max(wave_incl_max(own[lane]), carry);
      carry = lane_get(o, 63);
      const uint32_t g = st + lane;
      if (g < T) P.out_ids[dst_s[wv][o] + g] = stage[src_s[wv][o] + g];
    }
    __builtin_amdgcn_wave_barrier();
  }
}

static int lane_blocks_per_cu() {
  static int per_cu = 0;
  if (per_cu == 0 &&
      (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lane_kernel<LWAVES, false>, 64 * LWAVES, 0) != hipSuccess ||
       per_cu < 1))
    per_cu = 1;
  return per_cu;
}

}  // namespace tok6

hipError_t finish_lane_segment(TokParams P, const SplitParams& S, const tok6::LaneParams& Q, int n_cu, int fb_grid,
                               hipStream_t s);

hipError_t launch_tokenize_lane(const TokParams& P, int64_t nbytes, int64_t* tile_sent, SplitParams S,
                                tok6::LaneParams Q, const uint16_t* d_ctab, int n_cu, int fb_grid, hipStream_t s,
                                SplitTiming* tm) {
  if (tm) tm->n[0] = tm->n[1] = tm->n[2] = 0;
  auto mark = [&](int k, int side) -> hipError_t {
    if (!tm || tm->n[k] >= 64) return hipSuccess;
    const hipError_t e = hipEventRecord(tm->ev[k][side][tm->n[k]], s);
    if (side == 1) ++tm->n[k];
    return e;
  };
  const int64_t n_tiles = tile_count(nbytes);
  hipError_t e = launch_tile_bounds(P.sent_off, P.n_sent, n_tiles, tile_sent, const_cast<int64_t*>(S.tile_off), s);
  if (e != hipSuccess) return e;
  if ((e = hipMemsetAsync(P.out_tok_off, 0, sizeof(int64_t), s)) != hipSuccess) return e;
  S.tile_sent = tile_sent;
  Q.tile_sent = tile_sent;
  Q.tile_off = S.tile_off;
  Q.stage = S.ent;
  Q.ctr = S.chunk_ctr;
  Q.fb_list = S.fb_list;
  Q.fb_count = S.fb_count;
  Q.n_fallback = S.n_fallback;
  const int64_t seg = S.seg_tiles > 0 ? S.seg_tiles : SPLIT_SEG_TILES;
  const int grid = n_cu * tok6::lane_blocks_per_cu();
  const bool dbg = Q.stats && getenv("LDDL_LANE_STATS") && getenv("LDDL_LANE_STATS")[0] == '2';
  for (int64_t t0 = 0; t0 < n_tiles; t0 += seg) {
    S.t0 = Q.t0 = t0;
    S.t1 = Q.t1 = std::min(n_tiles, t0 + seg);
    Q.segb = t0 << 10;  // (+ sent_off[0], added on the device)
    if ((e = hipMemsetAsync(S.chunk_ctr, 0, 8, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(S.fb_count, 0, 4, s)) != hipSuccess) return e;
    if ((e = mark(0, 0)) != hipSuccess) return e;
    if (dbg)
      hipLaunchKernelGGL((tok6::lane_kernel<tok6::LWAVES, true>), dim3((unsigned)grid), dim3(64 * tok6::LWAVES), 0, s,
                         P, Q, d_ctab);
    else
      hipLaunchKernelGGL((tok6::lane_kernel<tok6::LWAVES, false>), dim3((unsigned)grid), dim3(64 * tok6::LWAVES), 0,
                         s, P, Q, d_ctab);
    if ((e = hipGetLastError()) != hipSuccess || (e = mark(0, 1)) != hipSuccess || (e = mark(2, 0)) != hipSuccess)
      return e;
    if ((e = finish_lane_segment(P, S, Q, n_cu, fb_grid, s)) != hipSuccess || (e = mark(2, 1)) != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t finish_lane_segment(TokParams P, const SplitParams& S, const tok6::LaneParams& Q, int n_cu, int fb_grid,
                               hipStream_t s) {
  TokParams F = P;
  F.out_ids = S.ent - (S.t0 << 10);  // the serial path writes at sent_off[s] - sent_off[0]
  hipError_t e = launch_tokenize_fallback(F, S.fb_list, S.fb_count, fb_grid, s);
  if (e != hipSuccess) return e;
  if ((e = launch_scan_ntok_range(P.out_ntok, S.tile_sent + S.t0, S.tile_sent + S.t1, S.seg_sent_cap, P.out_tok_off,
                                  S.scan_bsum, s)) != hipSuccess)
    return e;
  hipLaunchKernelGGL(tok6::compact_kernel, dim3((unsigned)std::max(1, n_cu * 16)), dim3(256), 0, s, P, Q.stage,
                     Q.segb, S.tile_sent, S.t0, S.t1);
  return hipGetLastError();
}

}  // namespace lddl
