// BERT NSP packing with one WAVE per partition (default packer).
//
// Same contract and results as pack_bert_kernel in pack.hip (reference:
// lddl/dask/bert/pretrain.py:241-365 create_pairs_from_document, :161-176
// _truncate_seq_pair, :386-402 _to_partition_pairs; binning.py:63-93), but
// the partition's serial decision chain runs out of LDS and uses the 64 lanes
// wherever the reference's loops are data-parallel:
//   * MT19937 state in LDS; the twist (in 64-word chunks, ascending -- the
//     in-place dependences of the sequential generator hold chunk-wise) and
//     the tempering run on all lanes; a draw is one LDS read.
//   * sentence filtering (drop empty sentences / documents) = wave scans.
//   * "accumulate sentences until len >= target" (chunk flush, random-next
//     B) = a wave prefix sum over the next 64 sentence lengths + ballot.
//   * _truncate_seq_pair: the side of every step is a closed form of the two
//     lengths, and random() < 0.5 <=> the first tempered word's MSB is 0, so
//     64 steps are decided per wave instruction (ballot + popcount).
//   * shuffle: Fisher-Yates on a u16 order array in LDS; binning: a stable
//     ballot partition per bin; token offsets: wave scan.
// Partitions larger than the LDS capacities (PW_*) run the same code with the
// arrays in global memory (wave-uniform branch).
#include "common.h"
#include "pack.h"
#include "wave.h"

#include <cmath>
#include <cstddef>
#include <cstdlib>
#include <type_traits>

namespace lddl {

// Per-partition arrays live in dynamic LDS sized by the host from the largest
// partition (PackParams cap_*); a partition that does not fit runs the same
// code on global memory (wave-uniform branch).
constexpr int PW_DOCS = 512;    // documents held in static LDS by the global-only variant
constexpr int PACK_OCC = 8;          // BERT packer held to 8 waves/SIMD (78 SGPRs; 7 at 106): pack 36.7 -> 35.6 ms
constexpr int PACK_DRAW_ROUNDS = 3;  // shuffle_draws: bound-propagation rounds before the ordered walk
struct PackWaveLds {
  uint32_t mt[MT_N];            // MT19937 state; draws temper on the fly
};
// global-only unmasked variant: the partition's documents (first kept slot
// relative to s0, #kept sentences) for the random-next lookups.  The masked
// variants read them from global memory: their LDS bounds the resident waves
// (mt + MaskLds), and the document lookups are a small part of their time.
struct PackDocLds {
  uint16_t dfirst[PW_DOCS];
  uint16_t dn[PW_DOCS];
};
struct PackDyn {                // views into the dynamic LDS region
  uint16_t* lens;               // [cap_lens] filtered sentence lengths
  uint16_t* dfirst;             // [cap_docs] relative to the partition's first slot
  uint16_t* dn;                 // [cap_docs]
  uint16_t* order;              // [cap_pairs] shuffle order
  uint16_t* ntk;                // [cap_pairs] num_tokens per pair record
  uint32_t* spec;               // [cap_lens / 32 + 2] (masking) slot holds a [CLS]/[SEP] token
};
extern __shared__ __attribute__((aligned(16))) uint8_t pw_dyn[];

// static masking lists (MASK instantiations only), sized for target_seq_length
// <= 512 with <= MLM_PICKS_1 picks per pair (MASK = 1) or <= MLM_MAX_SEQ
// (MASK = 2): the smaller lists leave LDS for more resident waves (MASK = 1:
// 4.5 KB with the MT state, 32 one-wave blocks per CU)
constexpr int MLM_PICKS_1 = 256;
template <int CAP, int PCAP>
struct MaskLds {
  alignas(16) uint16_t jb[CAP + 8];  // shuffle draws: swap x[i] <-> x[jb[i]]
  uint16_t mpos[PCAP];          // picked positions in pick order
  uint16_t mid[PCAP];           // their replacement ids (MLM_KEEP = unchanged)
};
struct NoMaskLds {};

size_t pack_dyn_bytes(int cap_lens, int cap_docs, int cap_pairs, bool mask) {
  return 2 * (size_t)cap_lens + 4 * (size_t)cap_docs + 4 * (size_t)cap_pairs + (mask ? 4 * (size_t)(cap_lens / 32 + 2) : 0);
}

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// global writes of this wave visible to its later reads (other lanes)
__device__ __forceinline__ void gsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ int wscan_incl(int v, int lane) {
  (void)lane;
  return wave_incl_add(v);
}

__device__ __forceinline__ int wsum(int v) { return lane_get(wave_incl_add(v), 63); }

// a wave-uniform value copied into a VGPR (v_mov): arithmetic on it runs on
// the vector unit -- for values only per-lane tests read
__device__ __forceinline__ int vgpr(int x) {
  int v;
  asm("v_mov_b32 %0, %1" : "=v"(v) : "s"(x));
  return v;
}

// popcount of a wave mask on the vector unit (two v_bcnt_u32_b32): the result
// is a VGPR value the scalar unit does not touch
__device__ __forceinline__ int vpopc64(uint64_t m) {
  int r;
  asm volatile("v_bcnt_u32_b32 %0, %1, 0\n\tv_bcnt_u32_b32 %0, %2, %0"
               : "=&v"(r)
               : "s"((uint32_t)m), "s"((uint32_t)(m >> 32)));
  return r;
}

typedef __attribute__((address_space(3))) uint32_t lds_u32;

// MT19937 twist (64-word chunks, ascending: the in-place dependences of the
// sequential generator hold chunk-wise), all lanes.  Out of
// line: every draw site would otherwise inline its own copy (code size, SGPR
// spills); LDS-qualified pointers keep it on ds_* instructions.
__device__ __attribute__((noinline)) void pack_mt_refill(lds_u32* mt, int lane) {
  for (int c = 0; c < MT_N; c += 64) {
    const int i = c + lane;
    uint32_t v = 0;
    if (i < MT_N) {
      const uint32_t a = mt[i], b = mt[i + 1 == MT_N ? 0 : i + 1];
      const uint32_t m = mt[i + MT_M >= MT_N ? i + MT_M - MT_N : i + MT_M];
      const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
      v = m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    wsync();
    if (i < MT_N) mt[i] = v;
    wsync();
  }
}

// ---- CPython MT19937 with the state in LDS -----------------------------
// init_by_array starts from init_genrand(19650218) whatever the seed: that
// state is a compile-time table
struct MtTable {
  uint32_t v[MT_N];
};
constexpr MtTable mt_genrand_table(uint32_t s) {
  MtTable t{};
  t.v[0] = s;
  for (int i = 1; i < MT_N; ++i) t.v[i] = 1812433253u * (t.v[i - 1] ^ (t.v[i - 1] >> 30)) + (uint32_t)i;
  return t;
}
__constant__ MtTable kMtGenrand = mt_genrand_table(19650218u);

// random.seed(seed + p) (CPython init_by_array, key = the seed's 32-bit words,
// klen <= 2), a LANE per partition: the whole corpus's seeding is one short
// launch (vs one serial chain per packer wave on the shared scalar unit).
// Each lane's 1247-step chain carries mt[i-1] in a register; its words go
// straight to the partition's 624-word row in global memory (the packer's
// coalesced load, WaveRng::load), and the second loop reads back what the
// first wrote there (independent of the chain, so the loads run ahead).
// Rows exist for every lane of the grid (the buffer is rounded up to 64
// partitions): no store guards.
__global__ __launch_bounds__(64) void mt_seed_states_kernel(uint64_t seed, uint32_t* __restrict__ states) {
  const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x;
  const uint64_t n = seed + (uint64_t)p;
  const uint32_t key0 = (uint32_t)n;
  const uint32_t key1 = (n >> 32) ? (uint32_t)(n >> 32) + 1u : key0;  // step k odd: key[k % klen] + k % klen
  uint32_t* const r = states + p * MT_N;
  // first loop, N steps from i = 1 over init_genrand(19650218)'s words: i =
  // 1..623, then mt[0] = mt[623] and i = 1 again
  uint32_t prev = kMtGenrand.v[0];
  prev = (kMtGenrand.v[1] ^ ((prev ^ (prev >> 30)) * 1664525u)) + key0;
  const uint32_t m1a = prev;
#pragma unroll 8
  for (int i = 2; i < MT_N; ++i) {
    prev = (kMtGenrand.v[i] ^ ((prev ^ (prev >> 30)) * 1664525u)) + ((i & 1) ? key0 : key1);
    r[i] = prev;
  }
  prev = (m1a ^ ((prev ^ (prev >> 30)) * 1664525u)) + key1;  // step N - 1 (odd), position 1
  const uint32_t m1 = prev;
  // second loop, N - 1 steps: i = 2..623, then position 1
#pragma unroll 8
  for (int i = 2; i < MT_N; ++i) {
    prev = (r[i] ^ ((prev ^ (prev >> 30)) * 1566083941u)) - (uint32_t)i;
    r[i] = prev;
  }
  r[1] = (m1 ^ ((prev ^ (prev >> 30)) * 1566083941u)) - 1u;
  r[0] = 0x80000000u;
}

hipError_t launch_mt_seed_states(uint64_t seed, int64_t n_part, uint32_t* states, hipStream_t s) {
  if (n_part < 1) return hipSuccess;
  hipLaunchKernelGGL(mt_seed_states_kernel, dim3((unsigned)((n_part + 63) / 64)), dim3(64), 0, s, seed, states);
  return hipGetLastError();
}

struct WaveRng {
  PackWaveLds& L;
  int lane;
  int idx;            // wave-uniform
  int wend = 0;       // tempered words [wend - 64, wend) (64-aligned) held in `win`, one per lane
                      // (one LDS read per 64 draws); draws below wend come from it
  uint32_t win = 0;

  // random.seed(seed + p): the state mt_seed_states_kernel left for this
  // partition (624 words, coalesced), the next draw twists
  __device__ __forceinline__ void load(const uint32_t* __restrict__ st) {
    for (int c = lane; c < MT_N; c += 64) L.mt[c] = st[c];
    wsync();
    idx = MT_N;
  }

  __device__ static __forceinline__ uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }

  // twist + temper on all lanes (out of line: pack_mt_refill)
  __device__ __forceinline__ void refill() {
    pack_mt_refill((lds_u32*)L.mt, lane);
    idx = 0;
    wend = 0;
  }

  // a draw: one compare on the fast path (the window ends at the state's end,
  // so idx < wend also means no twist is due)
  __device__ __forceinline__ uint32_t next() {
    if (idx >= wend) {
      if (idx >= MT_N) refill();
      const int wb = idx & ~63;  // windows start at multiples of 64
      wend = min(wb + 64, MT_N);
      win = temper(L.mt[min(wb + lane, MT_N - 1)]);
    }
    // v_readlane's lane select is its SGPR operand's bits [5:0]: with
    // 64-aligned windows the word at idx is lane idx & 63 (no offset math)
    return (uint32_t)__builtin_amdgcn_readlane((int)win, idx++);
  }
  // two consecutive words with one window test when both are in the window
  __device__ __forceinline__ void next2(uint32_t& a, uint32_t& b) {
    if (idx + 1 < wend) {
      a = (uint32_t)__builtin_amdgcn_readlane((int)win, idx);
      b = (uint32_t)__builtin_amdgcn_readlane((int)win, idx + 1);
      idx += 2;
    } else {
      a = next();
      b = next();
    }
  }
  __device__ __forceinline__ double random() {
    uint32_t a, b;
    next2(a, b);
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
  }
  // random() < 0.5  <=>  MSB of the first word is 0 (second word consumed)
  __device__ __forceinline__ bool coin_lt_half() {
    if (idx + 1 < wend) {
      const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)win, idx);
      idx += 2;
      return (a >> 31) == 0;
    }
    const uint32_t a = next();
    next();
    return (a >> 31) == 0;
  }
  __device__ __forceinline__ uint32_t randbelow(uint32_t n) {
    const int k = 32 - __clz(n);
    uint32_t r = next() >> (32 - k);
    while (r >= n) r = next() >> (32 - k);
    return r;
  }
  __device__ __forceinline__ int64_t randint(int64_t a, int64_t b) {
    return a + (int64_t)randbelow((uint32_t)(b - a + 1));
  }

  // random.shuffle's draws over m items (random.py shuffle: for q = m-1..1,
  // j = _randbelow(q+1)), recorded as jb[q] = j; the same words consumed as
  // m-1 sequential randbelow calls.  Wave-parallel over the next <= 64 MT
  // words: a batch covers the draws whose bounds n share one bit length k and
  // span <= 64 values [n_lo, n_hi], so each word's test r < n (r = word >> (32-k))
  // is already decided for every draw the batch could give it (r < n_lo:
  // accepted, r >= n_hi: rejected); only the words with r in [n_lo, n_hi) are
  // walked in order, one ballot step each.
  // REL: jb[q] holds j - (q & ~7) (signed 16-bit; the pick trace's chunk-relative form)
  template <bool REL = false, class T>
  __device__ __forceinline__ void shuffle_draws(int m, T* jb) { shuffle_draws_inl<REL>(m, jb); }
  template <bool REL = false, class T>
  __device__ __forceinline__ void shuffle_draws_inl(int m, T* jb) {
    int q = m - 1;
    while (q >= 1) {
      if (idx >= MT_N) refill();
      const int n_hi = q + 1;
      const int k = 32 - __clz((uint32_t)n_hi);
      const int n_lo = max(n_hi - 63, 1 << (k - 1));
      const int dmax = n_hi - n_lo + 1;  // draws this batch may complete (<= q)
      const int lim = min(MT_N - idx, 64);
      const uint64_t vm = lim >= 64 ? ~0ull : (1ull << lim) - 1ull;  // words before the state's end
      const uint32_t r = temper(L.mt[min(idx + lane, MT_N - 1)]) >> (32 - k);
      // (masks as wave-uniform values: every per-lane test of them below is
      // an exec mask or a v_mbcnt, no per-lane bit extraction)
      uint64_t accm = __ballot(r < (uint32_t)n_lo) & vm;
      uint64_t ambm = __ballot(r - (uint32_t)n_lo < (uint32_t)(n_hi - n_lo)) & vm;
      // bound propagation first: the words accepted before ambiguous word a
      // number at least L_a (decided accepts before a) and at most U_a (L_a +
      // undecided before a), so r < n_hi - U_a accepts it and r >= n_hi - L_a
      // rejects it.  Each round decides the first undecided word and, in
      // practice, most of the others: three rounds leave ~0.5 of a seq-512
      // shuffle's ~150 ambiguous words to the ordered walk below (simulated;
      // 1 / 2 / 3 rounds measured 2.11 / 1.91 / 1.87 e12 draw ticks per step).
#pragma unroll
      for (int it = 0; it < PACK_DRAW_ROUNDS; ++it) {
        if (!ambm) break;
        const int Lc = bits_below(accm);
        const int Uc = bits_below(ambm, Lc);
        // (r < 2^k <= 2^31 on the ambiguous lanes: no wrap there)
        const uint64_t acc_new = __ballot(r + (uint32_t)Uc < (uint32_t)n_hi) & ambm;
        const uint64_t rej_new = __ballot(r + (uint32_t)Lc >= (uint32_t)n_hi) & ambm;
        accm |= acc_new;
        ambm &= ~(acc_new | rej_new);
      }
      // a still-ambiguous word a (in order) is accepted iff the draws before
      // it, D_a decided + A earlier accepted ambiguous, leave its bound above
      // r: A < n_hi - r - D_a =: u_a.  Lanes past the batch's last draw are
      // resolved too and cut below (their outcome never feeds back).
      if (ambm) {
        const int u = n_hi - (int)r - bits_below(accm);
        int A = 0;
        while (ambm) {
          const int a = __ffsll((unsigned long long)ambm) - 1;
          ambm &= ambm - 1;
          const int ok = A < __builtin_amdgcn_readlane(u, a) ? 1 : 0;  // (scalar select, no branch)
          A += ok;
          accm |= (uint64_t)ok << a;
        }
      }
      const int pre = bits_below(accm);
      const uint64_t hit = __ballot(pre == dmax - 1) & accm;
      int end, s;
      if (hit) {
        end = __ffsll((unsigned long long)hit) - 1;
        s = dmax;
      } else {
        end = lim - 1;
        s = __popcll(accm);
      }
      if (lane_in(accm & (end >= 63 ? ~0ull : (2ull << end) - 1ull))) {
        const int qq = q - pre;
        jb[qq] = REL ? (T)((int)r - (qq & ~7)) : (T)r;
      }
      idx += end + 1;
      q -= s;
    }
    wsync();
  }

  // create_masked_lm_predictions' replacement choices for nm picks
  // (pretrain.py:224-232: random() < 0.8 -> [MASK]; else random() < 0.5 ->
  // keep; else vocab_words[randint(0, V-1)]), the same words consumed as the
  // sequential calls.  Every lane decides the pick that would start at its
  // word (its length 2 / 4 / 4 + randbelow's words and its id) from the next
  // <= 64 words; the walk from pick to pick is then read off jump tables.  A pick that
  // runs past the window starts the next window; one that cannot fit before
  // the state's end is drawn sequentially.
  __device__ __forceinline__ void mlm_choices(int nm, uint32_t V, uint32_t mask_id, uint32_t keep_id, uint16_t* mid) {
    const int kV = 32 - __clz(V);
    int pk = 0;
    while (pk < nm) {
      if (idx >= MT_N) refill();
      const int lim = min(MT_N - idx, 64);
      const uint32_t w = lane < lim ? temper(L.mt[idx + lane]) : 0u;
      // (the next two words by DPP wave shifts, not LDS permutes; lanes 62-63
      // read 0 there, and their picks need words past the window anyway)
      const uint32_t w1 = wave_shl1(w), w2 = wave_shl1(w1);
      const uint64_t accV = __ballot(lane < lim && (w >> (32 - kV)) < V);
      // random() < 0.8 on integers: random() = v * 2^-53 exactly, v = (w >> 5) * 2^26 + (w1 >> 6),
      // and 0.8 as a double is 7205759403792794 * 2^-53
      const bool lt08 = ((((uint64_t)(w >> 5)) << 26) | (uint64_t)(w1 >> 6)) < 7205759403792794ull;
      const uint64_t rest = lane + 4 < 64 ? accV & (~0ull << (lane + 4)) : 0ull;
      const int p = rest ? __ffsll((unsigned long long)rest) - 1 : 64;
      const uint32_t rv = (uint32_t)__shfl((int)(w >> (32 - kV)), p < 64 ? p : 63);
      bool res = false;
      int len = 0;
      uint32_t nid = 0;
      if (lane + 1 < lim && lt08) {
        res = true; len = 2; nid = mask_id;
      } else if (lane + 3 < lim && (w2 >> 31) == 0u) {
        res = true; len = 4; nid = keep_id;
      } else if (lane + 3 < lim && p < lim) {
        res = true; len = p - lane + 1; nid = rv;
      }
      const uint64_t resm = __ballot(res);
      int pos = 0;
      // the walk 0 -> nx[0] -> ... over resolved words (nx = l + len; it
      // stops at an unresolved word): lane d finds the walk's d-th word
      // c_d = nx^d(0) by the bits of d from jump tables J_i = nx^(2^i)
      // (J_{i+1} = J_i[J_i], one ds_bpermute each, built alongside the
      // walk's own gathers: ~5 dependent bpermutes per window, no LDS
      // stores or wave syncs).  len >= 2, so a window holds <= 32 picks,
      // and the members are a prefix of the lanes.  (A scalar walk cost ~10
      // scalar instructions per pick on the CU's one scalar unit; LDS-mark
      // pointer doubling 4 dependent LDS round trips per round.)
      if (resm & 1ull) {
        const int nx = res ? lane + len : 64;
        int J = min(nx, 64), c = 0;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          const int gc = __shfl(J, min(c, 63));  // J_i[c]
          const int gj = __shfl(J, min(J, 63));  // J_i[J_i]
          if ((lane >> i) & 1) c = c >= 64 ? 64 : gc;
          J = J >= 64 ? 64 : gj;
        }
        const bool member = lane < 32 && c < 64 && ((resm >> (c & 63)) & 1ull);
        const int cnt = min(__popcll(__ballot(member)), nm - pk);
        const uint32_t ng = (uint32_t)__shfl((int)nid, min(c, 63));
        if (lane < cnt) mid[pk + lane] = (uint16_t)ng;
        pos = __builtin_amdgcn_readlane(nx, __builtin_amdgcn_readlane(c, cnt - 1));
        pk += cnt;
      }
      if (pos == 0) {  // the pick does not fit before the state's end: sequential
        uint32_t v;
        if (random() < 0.8) v = mask_id;
        else if (random() < 0.5) v = keep_id;
        else v = randbelow(V);
        if (lane == 0) mid[pk] = (uint16_t)v;
        ++pk;
      } else {
        idx += pos;
      }
    }
    wsync();
  }
};

// random.shuffle(x) over x = order[0..np) (random.py: for i = n-1 .. 1,
// j = _randbelow(i+1), swap x[i], x[j]), order in global memory.  The draws
// first (shuffle_draws: the same MT words as the sequential calls) into
// scratch jq[q]; then the swaps in batches of 64 positions [qmin, qb]: the
// batch's slots -- its 64 positions (lane t = position qb - t) and the <= 64
// distinct positions below it that its draws hit -- are gathered into two
// registers per lane, the 64 swaps run in order on them (readlane +
// lane select), and the slots are scattered back.  Per 64 swaps: one coalesced
// read + write and <= 64 parallel gathers, where the swap loop paid a
// dependent global round trip per swap.
__device__ __forceinline__ void shuffle_global(WaveRng& rng, int np, int32_t* order, int32_t* jq, int lane) {
  rng.shuffle_draws_inl(np, jq);  // (inline: a call's clobbers cost the caller's SGPRs as spills)
  gsync();
  for (int qb = np - 1; qb >= 1; qb -= 64) {
    const int qmin = max(qb - 63, 1);
    const int q = qb - lane;
    const bool vq = q >= qmin;
    const int j = vq ? jq[q] : 0;
    int va = vq ? order[q] : 0;
    const bool low = vq && j < qmin;
    // the first lane whose draw hits the same position below the batch
    int first = 64;
    for (uint64_t m = __ballot(low); m;) {
      const int a = __ffsll((unsigned long long)m) - 1;
      const int ja = __builtin_amdgcn_readlane(j, a);
      const bool same = low && j == ja;
      if (same) first = a;
      m &= ~__ballot(same);
    }
    const bool own = low && first == lane;
    int vb = own ? order[j] : 0;
    const int sj = !vq ? lane : j >= qmin ? qb - j : 64 + first;  // slot of position j
    const int nq = qb - qmin + 1;
    for (int t = 0; t < nq; ++t) {
      const int s2 = __builtin_amdgcn_readlane(sj, t);
      const int x = __builtin_amdgcn_readlane(va, t);
      const int y = s2 < 64 ? __builtin_amdgcn_readlane(va, s2) : __builtin_amdgcn_readlane(vb, s2 - 64);
      va = lane == t ? y : va;
      if (s2 < 64) va = lane == s2 ? x : va;
      else vb = lane == s2 - 64 ? x : vb;
    }
    if (vq) order[q] = va;
    if (own) order[j] = vb;
    gsync();
  }
}

// binning reads the shuffled order once with each record's num_tokens packed
// in (rec | nt << 21; the record reads are random), then every bin pass
// reads it linearly
constexpr int PACKED_REC_BITS = 21;
__device__ __forceinline__ bool order_packable(int np, int max_seq) {
  return np < (1 << PACKED_REC_BITS) && max_seq < (1 << (32 - PACKED_REC_BITS));
}
__device__ __forceinline__ void pack_order_nt(int32_t* order, const PairRec* out, int np, int lane) {
  for (int k = lane; k < np; k += 64) {
    const int rec = order[k];
    order[k] = rec | ((int)out[rec].num_tokens << PACKED_REC_BITS);
  }
  gsync();
}

// smallest k in [k0, n) with (k == n-1) or (sum lens[k0..k] >= target);
// returns k and the sum.  lens via GET (LDS or global).  Positions past n
// read a length no target stops short of, so the first lane whose sum
// reaches the target, clamped to n - 1, is the answer (one compare per lane,
// no end-of-range masks on the scalar unit).
template <class GET>
__device__ __forceinline__ int find_fill(const GET& len_at, int k0, int n, int target, int lane, int* sum_out) {
  int base = 0;
  for (int k = k0; k < n; k += 64) {
    const int kk = k + lane;
    const int l = kk < n ? len_at(kk) : (1 << 20);
    const int ps = base + wscan_incl(l, lane);
    const uint64_t m = __ballot(ps >= target);
    if (m) {
      const int j = min((int)__builtin_ctzll(m), n - 1 - k);
      *sum_out = lane_get(ps, j);
      return k + j;
    }
    base = lane_get(ps, 63);
  }
  *sum_out = base;
  return n - 1;  // unreachable for n > 0
}

template <class GET>
__device__ __forceinline__ int range_sum(const GET& len_at, int k0, int k1, int lane) {
  int s = 0;
  for (int k = k0 + lane; k < k1; k += 64) s += len_at(k);
  return wsum(s);
}

// find_fill over a document of <= 64 sentences whose lengths' inclusive
// prefix sums are held one per lane in dps (lane k = sentence k, flat at the
// document total `tot` beyond it; one wave scan per document visit), dex the
// exclusive sums.  Lengths are >= 1 (kept sentences), so the sums rise
// strictly: the answer is the first lane whose sum reaches base + min(target,
// tot - base) (lane n - 1 when the target is out of reach), and lanes below
// k0 never do (the goal is >= base + 1).  One compare + one ballot, base
// returned for the A length (range_sum = dps[k1 - 1] - base).
__device__ __forceinline__ int find_fill_reg(int dps, int dex, int tot, int k0, int target, int* sum_out, int* base_out) {
  const int base = __builtin_amdgcn_readlane(dex, k0);
  const int vb = vgpr(base);  // (the goal on the vector unit: only the per-lane compare reads it)
  const int goal = vb + max(1, min(target, tot - vb));
  const int j = (int)__builtin_ctzll(__ballot(dps >= goal));
  *sum_out = __builtin_amdgcn_readlane(dps, j) - base;
  *base_out = base;
  return j;
}

// LDSOK = false: every LDS capacity is 0 (the default), the arrays are in
// global memory and the LDS/global branches compile away
// DBG: the phase stamps (LDDL_PACK_DEBUG=1) compiled in; the production
// instantiations carry no per-pair test of P.dbg on the scalar unit
template <int MASK, bool LDSOK, bool DBG>
__global__ __launch_bounds__(64, PACK_OCC) void pack_bert_wave_kernel(PackParams P) {
  __shared__ PackWaveLds L;
  __shared__ typename std::conditional<MASK != 0, MaskLds<MASK == 1 ? 512 : MLM_MAX_SEQ, MASK == 1 ? MLM_PICKS_1 : MLM_MAX_SEQ>, NoMaskLds>::type ML;
  __shared__ typename std::conditional<MASK != 0, NoMaskLds, PackDocLds>::type DL;
  PackDyn D;
  D.lens = reinterpret_cast<uint16_t*>(pw_dyn);
  D.dfirst = D.lens + P.cap_lens;
  D.dn = D.dfirst + P.cap_docs;
  D.order = D.dn + P.cap_docs;
  D.ntk = D.order + P.cap_pairs;
  D.spec = reinterpret_cast<uint32_t*>(D.ntk + P.cap_pairs);
  const int lane = threadIdx.x;
  const int64_t p = blockIdx.x;
  if (p >= P.n_part) return;
  const int64_t d0 = P.part_doc_off[p], d1 = P.part_doc_off[p + 1];
  const int64_t s0 = P.doc_sent_off[d0], s1 = P.doc_sent_off[d1];
  const int64_t pb = (int64_t)P.dup * s0;
  const int64_t base = P.sent_off[0];
  const int nsent = (int)(s1 - s0), ndoc = (int)(d1 - d0);
  // optional phase stamps (wave-uniform branch): filter, LDS fill, seed,
  // pair generation, shuffle, binning; masking: candidates, shuffle draws,
  // pick trace, 80/10/10 choices, sorted writes
  uint64_t ph[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, tprev = DBG ? __builtin_amdgcn_s_memtime() : 0;
  // (DBG: the wave's start and end on the 100 MHz device clock, for the
  // host's occupancy timeline: P.dbg[16 + 2p], [16 + 2p + 1])
  const uint64_t rt0 = DBG ? __builtin_amdgcn_s_memrealtime() : 0;
// generate sub-phases of the unmasked packer reuse the masking slots 6-10
#define PW_GSTAMP(k)                                    \
  if (!MASK && DBG) {                                   \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();   \
    ph[k] += t_ - tprev;                                \
    tprev = t_;                                         \
  }
#define PW_STAMP(k)                                     \
  if (DBG) {                                            \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();   \
    ph[k] += t_ - tprev;                                \
    tprev = t_;                                         \
  }

  // ---- filter: kept sentence slots via a running wave scan ---------------
  // kept_before[k] = #kept sentences before sentence s0 + k (k <= nsent)
  int32_t* kept_before = P.kept + s0 + p;
  // masking: does any kept sentence of the partition hold a [CLS] / [SEP]
  // token (literal specials in the text, rare)?  If none, every pair takes
  // the implicit candidate list with no per-pair flag reads
  bool part_spec = false;
  {
    int run = 0;
    for (int k = 0; k < nsent; k += 64) {
      const int kk = k + lane;
      int n = 0;
      if (kk < nsent) n = P.ntok[s0 + kk];
      const int keep = (kk < nsent && n > 0) ? 1 : 0;
      const int incl = wscan_incl(keep, lane);
      bool sp = false;
      if (kk < nsent) {
        const int slot = run + incl - keep;
        kept_before[kk] = slot;
        if (keep) {
          P.fs_ntok[s0 + slot] = (uint16_t)n;
          P.fs_base[s0 + slot] = P.sent_off[s0 + kk] - base;
          P.fs_dense[s0 + slot] = P.tokoff[s0 + kk];
          if (MASK) {
            const uint8_t f = P.sent_spec[s0 + kk];
            P.fs_spec[s0 + slot] = f;
            sp = f != 0;
          }
        }
      }
      if (MASK && __ballot(sp)) part_spec = true;
      run += lane_get(incl, 63);
    }
    if (lane == 0) kept_before[nsent] = run;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  // documents with >= 1 kept sentence, compacted
  int nd = 0;
  for (int k = 0; k < ndoc; k += 64) {
    const int kk = k + lane;
    int first = 0, cnt = 0;
    if (kk < ndoc) {
      const int a = (int)(P.doc_sent_off[d0 + kk] - s0), b = (int)(P.doc_sent_off[d0 + kk + 1] - s0);
      first = a < nsent ? kept_before[a] : kept_before[nsent];
      const int last = b < nsent ? kept_before[b] : kept_before[nsent];
      cnt = last - first;
    }
    const int keep = (kk < ndoc && cnt > 0) ? 1 : 0;
    const int incl = wscan_incl(keep, lane);
    if (keep) {
      const int di = nd + incl - 1;
      P.fd_first[d0 + di] = s0 + first;
      P.fd_n[d0 + di] = cnt;
    }
    nd += lane_get(incl, 63);
  }
  const int nfs = kept_before[nsent];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  PW_STAMP(0)
  const bool lres = LDSOK && nfs <= P.cap_lens && nd <= P.cap_docs;
  if (lres) {
    for (int k = lane; k < nfs; k += 64) D.lens[k] = (uint16_t)P.fs_ntok[s0 + k];
    for (int k = lane; k < nd; k += 64) {
      D.dfirst[k] = (uint16_t)(P.fd_first[d0 + k] - s0);
      D.dn[k] = (uint16_t)P.fd_n[d0 + k];
    }
    if constexpr (MASK) {
      for (int k = 0; k < nfs; k += 64) {
        const uint64_t m = __ballot(k + lane < nfs && P.fs_spec[s0 + k + lane] != 0);
        if (lane == 0) { D.spec[k >> 5] = (uint32_t)m; D.spec[(k >> 5) + 1] = (uint32_t)(m >> 32); }
      }
    }
  }
  wsync();
  PW_STAMP(1)
  // slot-relative accessors
  // global-only variant: the documents (the random-next lookups) in static LDS
  const bool dres = !MASK && !LDSOK && nd <= PW_DOCS && nfs < 65536;
  if constexpr (!MASK) {
    if (dres) {
      for (int k = lane; k < nd; k += 64) {
        DL.dfirst[k] = (uint16_t)(P.fd_first[d0 + k] - s0);
        DL.dn[k] = (uint16_t)P.fd_n[d0 + k];
      }
      wsync();
    }
  }
  auto len_at = [&](int k) -> int { return lres ? (int)D.lens[k] : P.fs_ntok[s0 + k]; };
  auto doc_first = [&](int d) -> int {
    if constexpr (!MASK) {
      if (dres) return (int)DL.dfirst[d];
    }
    return lres ? (int)D.dfirst[d] : (int)(P.fd_first[d0 + d] - s0);
  };
  auto doc_n = [&](int d) -> int {
    if constexpr (!MASK) {
      if (dres) return (int)DL.dn[d];
    }
    return lres ? (int)D.dn[d] : P.fd_n[d0 + d];
  };

  WaveRng rng{L, lane, MT_N};
  rng.load(P.mt_states + (int64_t)p * MT_N);
  PW_STAMP(2)
  const int max_num = P.max_seq - 3;
  PairRec* out = P.pairs + pb;
  int np = 0;
  int err = PACK_OK;
  const int pcap = P.cap_pairs;
  int64_t mcur = 0, mend = 0;  // this partition's current arena chunk
  int nmask_part = 0;
  (void)mcur; (void)mend; (void)nmask_part;
  // any filtered slot in [k0, k0 + n) holding a [CLS]/[SEP] token
  auto any_spec = [&](int k0, int n) -> bool {
    bool f = false;
    if constexpr (MASK) {
      if (!part_spec) return false;
      for (int k = 0; k < n; k += 64) {
        const int kk = k0 + k + lane;
        bool x = false;
        if (k + lane < n) x = lres ? ((D.spec[kk >> 5] >> (kk & 31)) & 1u) != 0 : P.fs_spec[s0 + kk] != 0;
        if (__ballot(x)) { f = true; break; }
      }
    }
    return f;
  };
  // a document of <= 64 sentences keeps its lengths in a register, loaded
  // one document visit ahead (the load flies while this visit's pairs run)
  // (with the document's first slot and length, carried to its visit)
  int df_next = 0, dn_next = 0;
  auto doc_lens = [&](int d) -> int {
    bool got = false;
    if constexpr (!MASK) {
      if (dres) {  // (one residence branch for both fields)
        df_next = (int)DL.dfirst[d];
        dn_next = (int)DL.dn[d];
        got = true;
      }
    }
    if (!got) {
      df_next = doc_first(d);
      dn_next = doc_n(d);
    }
    return dn_next <= 64 && lane < dn_next ? len_at(df_next + lane) : 0;
  };
  int dl_next = nd > 0 ? doc_lens(0) : 0;
  // the records of the current 64 pairs, one per lane (lane k = pair
  // (np & ~63) + k), written by one coalesced flush per 64 pairs: each pair's
  // fields are selected into these columns by the vector unit instead of
  // being packed, addressed and stored by lane 0 from scalar registers
  int c_fs0 = 0, c_fs1 = 0, c_lo0 = 0, c_hi0 = 0, c_lo1 = 0, c_hi1 = 0, c_n0 = 0, c_n1 = 0, c_rn = 0;
  auto flush = [&](int b, int cnt) {
    if (lane < cnt) {
      PairRec q;
      q.fs0 = s0 + c_fs0;
      q.fs1 = s0 + c_fs1;
      q.lo0 = (uint16_t)c_lo0; q.hi0 = (uint16_t)c_hi0;
      q.lo1 = (uint16_t)c_lo1; q.hi1 = (uint16_t)c_hi1;
      q.n0 = (uint16_t)c_n0; q.n1 = (uint16_t)c_n1;
      q.flags = (uint16_t)(c_rn | 2);
      q.num_tokens = (uint16_t)((c_hi0 - c_lo0) + (c_hi1 - c_lo1) + 3);
      out[b + lane] = q;
      if (b + lane < pcap) D.ntk[b + lane] = q.num_tokens;
    }
  };
  for (int dup = 0; dup < P.dup && !err; ++dup) {
    for (int di = 0; di < nd && !err; ++di) {
      const int first = df_next, len = dn_next;  // doc_first(di), doc_n(di) from the prefetch
      const bool dreg = len <= 64;
      const int dl = dl_next;
      const int dps = dreg ? wave_incl_add(dl) : 0;  // (dl is 0 past the document)
      const int dex = dps - dl;
      const int dtot = dreg ? __builtin_amdgcn_readlane(dps, 63) : 0;  // (flat past the document)
      if (di + 1 < nd) dl_next = doc_lens(di + 1);
      else if (dup + 1 < P.dup) dl_next = doc_lens(0);
      int target = max_num;
      if (rng.random() < P.short_seq_prob) target = (int)rng.randint(2, max_num);
      PW_GSTAMP(6)
      int i = 0;
      while (i < len) {
        const int cs = i;
        int cur;
        int fbase = 0;
        const int j = dreg ? find_fill_reg(dps, dex, dtot, cs, target, &cur, &fbase)
                           : find_fill([&](int k) { return len_at(first + k); }, cs, len, target, lane, &cur);
        const int nchunk = j - cs + 1;
        int a_end = 1;
        if (nchunk >= 2) a_end = (int)rng.randint(1, nchunk - 1);
        const int la = a_end == nchunk ? cur
                       : dreg ? __builtin_amdgcn_readlane(dps, cs + a_end - 1) - fbase
                              : range_sum([&](int k) { return len_at(first + k); }, cs, cs + a_end, lane);
        PW_GSTAMP(7)
        PairRec r;
        r.fs0 = s0 + first + cs;
        r.n0 = (uint16_t)a_end;
        int lb;
        bool rn;
        int i_next;
        if (nchunk == 1 || rng.coin_lt_half()) {
          rn = true;
          const int tb = target - la;
          // up to 10 draws for a document other than di (the first one almost always)
          int rdi = (int)rng.randbelow((uint32_t)nd);
          if (rdi == di) {
            for (int t = 1; t < 10 && rdi == di; ++t) rdi = (int)rng.randbelow((uint32_t)nd);
            if (rdi == di) rn = false;
          }
          int rfirst, rlen;  // (one branch on the table's residence for both fields)
          bool rdone = false;
          if constexpr (!MASK) {
            if (dres) {
              rfirst = (int)DL.dfirst[rdi];
              rlen = (int)DL.dn[rdi];
              rdone = true;
            }
          }
          if (!rdone) {
            rfirst = doc_first(rdi);
            rlen = doc_n(rdi);
          }
          // a document of <= 64 sentences: its lengths are loaded before
          // rstart is drawn (the load flies during the draw), then the fill
          // from rstart is one scan + one compare per lane (lengths >= 1:
          // the sums from rstart rise strictly, lanes below rstart hold 0)
          const bool rreg = rlen <= 64;
          const int rl = rreg && lane < rlen ? len_at(rfirst + lane) : 0;
          const int rstart = (int)rng.randint(0, rlen - 1);
          int k;
          if (rreg) {
            const int ps = wave_incl_add(lane >= rstart ? rl : 0);
            const int vt = vgpr(lane_get(ps, 63));
            k = (int)__builtin_ctzll(__ballot(ps >= max(1, min(tb, vt))));
            lb = lane_get(ps, k);
          } else {
            k = find_fill([&](int q) { return len_at(rfirst + q); }, rstart, rlen, tb, lane, &lb);
          }
          r.fs1 = s0 + rfirst + rstart;
          r.n1 = (uint16_t)(k - rstart + 1);
          i_next = j - (nchunk - a_end) + 1;
        } else {
          rn = false;
          lb = cur - la;
          r.fs1 = s0 + first + cs + a_end;
          r.n1 = (uint16_t)(nchunk - a_end);
          i_next = j + 1;
        }
        PW_GSTAMP(8)
        // _truncate_seq_pair, 64 steps per round.  Step t trims A while
        // t < th when A starts longer (pos), B while t < th otherwise, then
        // the sides alternate: side_a(t) = t < th ? pos : odd(t - th) == pos
        int alo = 0, ahi = la, blo = 0, bhi = lb;
        int E = la + lb - max_num;
        int t0 = 0;
        // (th / pos on the vector unit: only the per-lane side test reads them)
        const int d0l = vgpr(la) - lb;
        const int posi = d0l > 0 ? 1 : 0;
        const int th = posi ? d0l : 1 - d0l;
        auto side_a = [&](int t) -> bool { return (t < th ? posi : (((t - th) & 1) ^ posi ^ 1)) != 0; };
        auto trunc_round = [&](int n) {
          const uint64_t act = __ballot(lane < n);
          const int t = t0 + lane;
          const int sbit = t < th ? posi : (((t - th) & 1) ^ posi ^ 1);  // 1: this step trims A
          const int w = (int)WaveRng::temper(L.mt[min(rng.idx + 2 * lane, MT_N - 1)]);
          const uint64_t SA = __ballot(sbit != 0) & act, F = __ballot(w >= 0) & act;  // front: MSB 0
          // (the counts on the vector unit: the segment bounds then live in
          // VGPRs, where the record columns take them; the CU's one scalar
          // unit is the packer's bound)
          const int x = vpopc64(SA & F), a = vpopc64(SA), f = vpopc64(F);
          alo += x;
          ahi -= a - x;
          blo += f - x;
          bhi -= n - a - f + x;
          rng.idx += 2 * n;
          t0 += n;
          E -= n;
        };
        if (E > 0 && E <= 64 && 2 * E <= MT_N - rng.idx) {
          trunc_round(E);  // (the common case: one round, no loop)
        } else {
          while (E > 0) {
            const int avail = (MT_N - rng.idx) >> 1;
            if (avail == 0) {  // a step straddles the twist: one serial step
              const bool sideA = side_a(t0);
              const bool front = rng.coin_lt_half();
              if (sideA) { if (front) ++alo; else --ahi; } else { if (front) ++blo; else --bhi; }
              ++t0;
              --E;
              continue;
            }
            trunc_round(min(min(E, 64), avail));
          }
        }
        PW_GSTAMP(9)
        if (__builtin_amdgcn_readfirstlane((ahi - alo < 1 || bhi - blo < 1) ? 1 : 0)) { err = PACK_EASSERT; break; }
        if constexpr (MASK != 0) {  // (the masking code wants them uniform)
          alo = __builtin_amdgcn_readfirstlane(alo);
          ahi = __builtin_amdgcn_readfirstlane(ahi);
          blo = __builtin_amdgcn_readfirstlane(blo);
          bhi = __builtin_amdgcn_readfirstlane(bhi);
        }
        r.lo0 = (uint16_t)alo; r.hi0 = (uint16_t)ahi;
        r.lo1 = (uint16_t)blo; r.hi1 = (uint16_t)bhi;
        r.flags = (uint16_t)((rn ? 1 : 0) | 2);
        r.num_tokens = (uint16_t)((ahi - alo) + (bhi - blo) + 3);
        int64_t mref = 0;
        if constexpr (MASK) {
          // ---- create_masked_lm_predictions (pretrain.py:182-238) ----------
          PW_STAMP(3)
          const int la2 = ahi - alo, lb2 = bhi - blo;
          const int ntp = max(1, (int)rint((double)(la2 + lb2 + 3) * P.mlm_ratio));
          const int fa = first + cs, fb = (int)(r.fs1 - s0);
          const bool expl = any_spec(fa, a_end) || any_spec(fb, r.n1);
          // explicit candidate positions (pairs holding [CLS]/[SEP] tokens,
          // rare): global scratch of this partition, keeping the LDS lists
          // small for more resident waves
          uint16_t* const mcand = P.mcand + p * MLM_MAX_SEQ;
          int m = la2 + lb2;
          if (expl) {  // candidates = positions whose token is not [CLS]/[SEP]
            m = 0;
            auto seg = [&](int fs, int ns, int lo, int hi, int pos0) {
              int acc = 0;
              for (int q = 0; q < ns && acc < hi; ++q) {
                const int ln = len_at(fs + q);
                const int64_t sb = P.fs_dense[s0 + fs + q];
                const int a0 = max(lo, acc), a1 = min(hi, acc + ln);
                for (int t = a0; t < a1; t += 64) {
                  const int tt = t + lane;
                  bool keep = false;
                  if (tt < a1) {
                    const uint32_t v = P.ids[sb + (tt - acc)];
                    keep = v != P.cls_id && v != P.sep_id;
                  }
                  const uint64_t bm = __ballot(keep);
                  if (keep) mcand[m + bits_below(bm)] = (uint16_t)(pos0 + tt - lo);
                  m += __popcll(bm);
                }
                acc += ln;
              }
            };
            seg(fa, a_end, alo, ahi, 1);
            seg(fb, r.n1, blo, bhi, 2 + la2);
            gsync();  // the list's global writes visible to the trace's reads (other lanes)
          }
          // random.shuffle(cand_indexes): record the swaps, then undo them
          // per picked slot (lane per pick) instead of permuting the list
          PW_STAMP(6)
          rng.shuffle_draws<true>(m, ML.jb);
          PW_STAMP(7)
          const int nm = min(ntp, m);
          // pick pk's candidate = the slot that the swaps (q, jb[q]), applied
          // for q = m-1 .. 1, move to pk: traced back over q = 1 .. m-1.
          // Picks pk, pk + 64 per lane; 8 swaps per 16-B LDS read (measured
          // against u16 reads / readlane swaps: 2.87 vs 3.82 / 3.23 s per step)
          auto pick_pos = [&](int q) { return (uint16_t)(expl ? (int)mcand[q] : (q < la2 ? 1 + q : 2 + q)); };
          // Final position pk < nm of the shuffled list = the element the
          // swaps move there.  Split the swaps at nm: the late ones
          // (q = nm-1 .. 1, all j_q <= q < nm) only permute positions < nm
          // and are traced back per pick (lane per pick, O(nm)); the early
          // ones (q >= nm) only move elements INTO positions < nm: the element
          // at v < nm after them is found by successor chains -- F[v] = the
          // smallest q >= nm with j_q = v (the last early swap writing v), then
          // F[q] = the smallest q' > q with j_q' = q, ... until no swap wrote
          // the position (its original element).  F is u16 over the mpos + mid
          // lists (unused until the picks are known), built in chunks of 64
          // swaps from the last down: a later chunk's smaller q overwrite, and
          // lanes of one chunk on the same j store again until the smallest
          // stands (LDS has no 16-bit min; collisions are rare).
          constexpr int MCAP = MASK == 1 ? 512 : MLM_MAX_SEQ;
          const int nm8 = (nm + 7) & ~7;
          const bool split = nm < m && nm8 + nm <= MCAP;
          const int tr8 = split ? nm8 : (m + 7) & ~7;  // the traced swaps: [1, tr8)
          if (split) {
            uint16_t* F = ML.mpos;
            using MLT = std::remove_reference_t<decltype(ML)>;
            static_assert(offsetof(MLT, mid) == offsetof(MLT, mpos) + sizeof(ML.mpos), "mid follows mpos");
            static_assert(sizeof(ML.mpos) + sizeof(ML.mid) >= 2 * MCAP, "F spans mpos + mid");
            for (int k = lane; k < m; k += 64) F[k] = 0xFFFFu;
            wsync();
            PW_STAMP(8)  // (trace sub-phases: the list reset above -> m_trace; F build -> 11, chains -> 12)
            for (int qb = nm + ((m - nm - 1) & ~63); qb >= nm; qb -= 64) {
              const int q = qb + lane;
              uint32_t j = 0;
              bool pend = false;
              if (q < m) {
                j = (uint32_t)((int)(int16_t)ML.jb[q] + (q & ~7));
                pend = (uint32_t)q > j;
              }
              while (__ballot(pend) != 0) {
                if (pend) F[j] = (uint16_t)q;
                wsync();
                if (pend) pend = (uint32_t)F[j] > (uint32_t)q;
                wsync();
              }
            }
            PW_STAMP(11)
            // element at v after the early swaps -> jb[nm8 + v]
            for (int v = lane; v < nm; v += 64) {
              uint32_t val = (uint32_t)v, t = F[v];
              while (t != 0xFFFFu) {
                val = t;
                t = F[t];
              }
              ML.jb[nm8 + v] = (uint16_t)val;
            }
            PW_STAMP(12)
          }
          {
            // identity swaps pad the traced list: jb[0] = 0, jb[q] = q for q in
            // [end, tr8) (chunk-relative: q & 7)
            const int end = split ? nm : m;
            if (lane == 0) ML.jb[0] = 0;
            if (end + lane < tr8) ML.jb[end + lane] = (uint16_t)((end + lane) & 7);
            wsync();
            const uint4* jb4 = reinterpret_cast<const uint4*>(ML.jb);
            auto elem = [&](int q) { return split ? (int)ML.jb[nm8 + q] : q; };
            // one pick per lane, 64 picks per pass: swaps below a pass's first
            // pick leave its picks in place, so pass k traces [64k, tr8)
            for (int pb0 = 0; pb0 < nm; pb0 += 64) {
              const int pk = pb0 + lane;
              // chunk-relative: d = qa - c against swap (t, j - c), t and the
              // chunk's j - c as stored: no per-swap index materialisation
              int d = pk - pb0;
              for (int c = pb0; c < tr8; c += 8) {
                const uint4 w = jb4[c >> 3];
                const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                  const int jc = (t & 1) ? (int)ww[t >> 1] >> 16 : (int)(int16_t)(ww[t >> 1] & 0xFFFFu);
                  d = d == t ? jc : (d == jc ? t : d);
                }
                d -= 8;
              }
              const int qa = d + tr8;
              const int ea = pk < nm ? elem(qa) : 0;
              wsync();  // (mpos overlaps F: every lane has read its chains)
              if (pk < nm) ML.mpos[pk] = pick_pos(ea);
            }
          }
          // 80% [MASK], 10% keep, 10% random word, in pick order
          PW_STAMP(8)
          rng.mlm_choices(nm, P.n_vocab, P.mask_id, MLM_KEEP, ML.mid);
          PW_STAMP(9)
          if (mcur + nm > mend) {
            unsigned long long b0 = 0;
            if (lane == 0) b0 = atomicAdd(P.mcounter, (unsigned long long)MLM_CHUNK);
            mcur = (int64_t)__shfl((long long)b0, 0);
            mend = mcur + MLM_CHUNK;
          }
          const bool fits = (uint64_t)mend <= P.mcap;
          // sorted(masked_lms) by position: the picks are distinct positions
          // < MCAP, so a pick's rank = the set bits below it in a position
          // bitmap (jb is free after the trace): per-dword prefix counts
          // by one wave scan, then two LDS reads per pick
          {
            constexpr int NW = MCAP / 32;
            static_assert(2 * NW <= MCAP / 2, "bitmap + prefix counts fit in jb");
            uint32_t* bm = reinterpret_cast<uint32_t*>(ML.jb);
            uint32_t* pre = bm + NW;
            for (int w = lane; w < NW; w += 64) bm[w] = 0;
            wsync();
            for (int pk = lane; pk < nm; pk += 64) {
              const uint32_t pos = ML.mpos[pk];
              atomicOr(&bm[pos >> 5], 1u << (pos & 31));
            }
            wsync();
            uint32_t carry = 0;
            for (int w0 = 0; w0 < NW; w0 += 64) {
              const uint32_t c = w0 + lane < NW ? (uint32_t)__popc(bm[w0 + lane]) : 0u;
              const uint32_t x = wave_incl_add(c);
              if (w0 + lane < NW) pre[w0 + lane] = carry + x - c;
              carry += lane_get(x, 63);
            }
            wsync();
            for (int pk = lane; pk < nm; pk += 64) {
              if (!fits) break;
              const uint32_t pos = ML.mpos[pk];
              const int rank = (int)(pre[pos >> 5] + __popc(bm[pos >> 5] & ((1u << (pos & 31)) - 1u)));
              P.marena[mcur + rank] = pos | ((uint32_t)ML.mid[pk] << 16);
            }
          }
          mref = mcur | ((int64_t)nm << 48);
          mcur += nm;
          wsync();
          PW_STAMP(10)
        }
        {
          const bool me = lane == (np & 63);
          c_fs0 = me ? (int)(r.fs0 - s0) : c_fs0;
          c_fs1 = me ? (int)(r.fs1 - s0) : c_fs1;
          c_lo0 = me ? alo : c_lo0;
          c_hi0 = me ? ahi : c_hi0;
          c_lo1 = me ? blo : c_lo1;
          c_hi1 = me ? bhi : c_hi1;
          c_n0 = me ? (int)r.n0 : c_n0;
          c_n1 = me ? (int)r.n1 : c_n1;
          c_rn = me ? (rn ? 1 : 0) : c_rn;
        }
        if (MASK && lane == 0) P.mref[pb + np] = mref;
        ++np;
        if ((np & 63) == 0) flush(np - 64, 64);
        i = i_next;
        PW_GSTAMP(10)
      }
    }
  }
  if (!err && (np & 63)) flush(np & ~63, np & 63);
  PW_STAMP(3)
  if (lane == 0) P.part_err[p] = err;
  if (err) {
    if (lane == 0) { P.part_npairs[p] = 0; P.part_ntok[p] = 0; if (MASK) P.part_nmask[p] = 0; }
    return;
  }
  wsync();
  // ---- random.shuffle(partition_pairs) -----------------------------------
  const bool ores = LDSOK && np <= pcap;
  int32_t* gorder = P.order + pb;
  if (ores) for (int k = lane; k < np; k += 64) D.order[k] = (uint16_t)k;
  else for (int k = lane; k < np; k += 64) gorder[k] = k;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  if (ores) {
    // lane 0 alone touches the order array here (program order suffices)
    for (int k = np - 1; k >= 1; --k) {
      const int j = (int)rng.randbelow((uint32_t)(k + 1));
      if (lane == 0) { const uint16_t t = D.order[k]; D.order[k] = D.order[j]; D.order[j] = t; }
    }
  } else {
    shuffle_global(rng, np, gorder, P.binned + pb, lane);  // (binned: draw scratch until binning)
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  PW_STAMP(4)
  const bool packed = !ores && order_packable(np, P.max_seq);
  if (packed) pack_order_nt(gorder, out, np, lane);
  auto ord_at = [&](int k) -> int { return ores ? (int)D.order[k] : packed ? gorder[k] & ((1 << PACKED_REC_BITS) - 1) : gorder[k]; };
  auto ntk_at = [&](int k, int rec) -> int {
    return ores ? (int)D.ntk[rec] : packed ? (int)((uint32_t)gorder[k] >> PACKED_REC_BITS) : (int)out[rec].num_tokens;
  };
  // ---- stable bin partition + token offsets -------------------------------
  const int nb = P.nbins;
  int32_t* binned = P.binned + pb;
  int64_t* tl = P.tok_local + pb;
  int pos = 0;
  int64_t acc = 0, macc = 0;
  for (int b = 0; b < nb; ++b) {
    int cnt = 0;
    for (int k = 0; k < np; k += 64) {
      const int kk = k + lane;
      int rec = 0, nt = 0;
      bool in = false;
      if (kk < np) {
        rec = ord_at(kk);
        nt = ntk_at(kk, rec);
        int bb = (nt - 1) / P.bin_size;
        bb = bb > nb - 1 ? nb - 1 : bb;
        in = bb == b;
      }
      const uint64_t m = __ballot(in);
      const int before = __popcll(m & ((1ull << lane) - 1ull));
      const int tinc = wscan_incl(in ? nt : 0, lane);
      if (in) {
        binned[pos + before] = rec;
        tl[pos + before] = acc + tinc - nt;
      }
      if constexpr (MASK) {
        const int nmk = in ? (int)((uint64_t)P.mref[pb + rec] >> 48) : 0;
        const int minc = wscan_incl(nmk, lane);
        if (in) P.mloc[pb + pos + before] = macc + minc - nmk;
        macc += lane_get(minc, 63);
      }
      pos += __popcll(m);
      cnt += __popcll(m);
      acc += lane_get(tinc, 63);
    }
    if (lane == 0) P.bin_count[p * nb + b] = cnt;
  }
  if (lane == 0) {
    P.part_npairs[p] = np;
    P.part_ntok[p] = acc;
    if (MASK) P.part_nmask[p] = macc;
  }
  PW_STAMP(5)
  if (DBG && lane == 0) {
    for (int k = 0; k < 6; ++k) atomicAdd((unsigned long long*)&P.dbg[k], (unsigned long long)ph[k]);
    atomicAdd((unsigned long long*)&P.dbg[6], (unsigned long long)np);
    atomicAdd((unsigned long long*)&P.dbg[7], 1ull);
    for (int k = 6; k < 14; ++k) atomicAdd((unsigned long long*)&P.dbg[k + 2], (unsigned long long)ph[k]);
    P.dbg[16 + 2 * p] = rt0;
    P.dbg[16 + 2 * p + 1] = __builtin_amdgcn_s_memrealtime();
  }
#undef PW_STAMP
#undef PW_GSTAMP
}

// LDDL_PACK_WAVES_CU=w (occupancy experiments): dynamic LDS padded so that at
// most w of the kernel's one-wave blocks fit on a CU (160 KiB LDS)
static size_t occupancy_pad(const void* fn, size_t dyn) {
  const char* e = getenv("LDDL_PACK_WAVES_CU");
  const int w = e ? atoi(e) : 0;
  hipFuncAttributes a;
  if (w <= 0 || hipFuncGetAttributes(&a, fn) != hipSuccess) return dyn;
  const size_t per = (size_t)160 * 1024 / (size_t)(w + 1) + 512;  // > 1/(w+1) of the LDS per block
  return per > a.sharedSizeBytes + dyn ? per - a.sharedSizeBytes : dyn;
}

hipError_t launch_pack_bert_wave(const PackParams& P, hipStream_t s) {
  const size_t dyn0 = pack_dyn_bytes(P.cap_lens, P.cap_docs, P.cap_pairs, P.masking != 0);
  const bool lds = P.cap_lens > 0 || P.cap_docs > 0 || P.cap_pairs > 0;
  const dim3 g((unsigned)P.n_part), b(64);
#define PW_LAUNCH(M, L)                                                                                  \
  do {                                                                                                   \
    if (P.dbg) {                                                                                         \
      const size_t dyn = occupancy_pad((const void*)pack_bert_wave_kernel<M, L, true>, dyn0);           \
      hipLaunchKernelGGL((pack_bert_wave_kernel<M, L, true>), g, b, dyn, s, P);                         \
    } else {                                                                                             \
      const size_t dyn = occupancy_pad((const void*)pack_bert_wave_kernel<M, L, false>, dyn0);          \
      hipLaunchKernelGGL((pack_bert_wave_kernel<M, L, false>), g, b, dyn, s, P);                        \
    }                                                                                                    \
  } while (0)
  // (every pair's picks: max(1, rint(num_tokens * ratio)), num_tokens <= max_seq)
  if (P.masking && P.max_seq <= 512 && std::max(1, (int)rint((double)P.max_seq * P.mlm_ratio)) <= MLM_PICKS_1) {
    if (lds) PW_LAUNCH(1, true);
    else PW_LAUNCH(1, false);
  } else if (P.masking) {
    if (lds) PW_LAUNCH(2, true);
    else PW_LAUNCH(2, false);
  } else {
    if (lds) PW_LAUNCH(0, true);
    else PW_LAUNCH(0, false);
  }
#undef PW_LAUNCH
  return hipGetLastError();
}

// ------------------------------------------------------------- CodeBERT ----
// pretrain_codebert.py:343-442 create_pairs_from_document + :236-247
// _truncate_seq, one wave per partition (same contract and results as
// pack_codebert_kernel in pack.hip, the lane-serial variant).  The serial
// "accumulate segments until the chunk overflows" loops become wave prefix
// sums + ballots, _truncate_seq decides 64 coins per round, the shuffle /
// binning are the BERT wave packer's (global-memory arrays).

// smallest k in [k0, n) with (k == stop) or (base + sum lens[k0..k] > limit);
// returns -1 (and the total in *sum_out) when there is none
template <class GET>
__device__ __forceinline__ int find_over(const GET& len_at, int k0, int n, int stop, int base, int limit, int lane,
                                         int* sum_out) {
  for (int k = k0; k < n; k += 64) {
    const int kk = k + lane;
    const int l = kk < n ? len_at(kk) : 0;
    const int ps = base + wscan_incl(l, lane);
    const uint64_t m = __ballot(kk < n && (kk == stop || ps > limit));
    if (m) {
      const int j = __ffsll((unsigned long long)m) - 1;
      *sum_out = lane_get(ps, j);
      return k + j;
    }
    base = lane_get(ps, 63);
  }
  *sum_out = base;
  return -1;
}

// _truncate_seq on [lo, hi) down to max_n tokens: one coin (= one random()
// call, 2 MT words) per excess token, MSB of the first word decides
__device__ __forceinline__ void trunc_seq_wave(WaveRng& rng, PackWaveLds& L, int lane, int& lo, int& hi, int max_n) {
  int E = (hi - lo) - max_n;
  while (E > 0) {
    const int avail = (MT_N - rng.idx) >> 1;
    if (avail == 0) {  // a coin straddles the twist: one serial step
      if (rng.coin_lt_half()) ++lo; else --hi;
      --E;
      continue;
    }
    const int n = min(min(E, 64), avail);
    const bool act = lane < n;
    const bool front = act ? (WaveRng::temper(L.mt[rng.idx + 2 * lane]) >> 31) == 0 : false;
    const int f = __popcll(__ballot(front));  // (front is false past the n steps)
    lo += f;
    hi -= n - f;
    rng.idx += 2 * n;
    E -= n;
  }
}

__global__ __launch_bounds__(64) void pack_codebert_wave_kernel(PackParams P) {
  __shared__ PackWaveLds L;
  const int lane = threadIdx.x;
  const int64_t p = blockIdx.x;
  if (p >= P.n_part) return;
  const int64_t d0 = P.part_doc_off[p], d1 = P.part_doc_off[p + 1];
  const int64_t s0 = P.doc_sent_off[d0], s1 = P.doc_sent_off[d1];
  const int64_t pb = (int64_t)P.dup * s0;
  const int64_t base = P.sent_off[0];
  const int nsent = (int)(s1 - s0), ndoc = (int)(d1 - d0);
  // ---- filter: kept segment slots (wave scan), kept documents ------------
  int32_t* kept_before = P.kept + s0 + p;
  {
    int run = 0;
    for (int k = 0; k < nsent; k += 64) {
      const int kk = k + lane;
      const int n = kk < nsent ? P.ntok[s0 + kk] : 0;
      const int keep = (kk < nsent && n > 0) ? 1 : 0;
      const int incl = wscan_incl(keep, lane);
      if (kk < nsent) {
        const int slot = run + incl - keep;
        kept_before[kk] = slot;
        if (keep) {
          P.fs_ntok[s0 + slot] = (uint16_t)n;
          P.fs_base[s0 + slot] = P.sent_off[s0 + kk] - base;
          P.fs_dense[s0 + slot] = P.tokoff[s0 + kk];
        }
      }
      run += lane_get(incl, 63);
    }
    if (lane == 0) kept_before[nsent] = run;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  // a document is kept when it has a kept code segment (len(CodePair) > 0,
  // pretrain_codebert.py:161); its first fd_nd kept slots are docstring
  int nd_docs = 0;
  for (int k = 0; k < ndoc; k += 64) {
    const int kk = k + lane;
    int first = 0, cnt = 0, ndseg = 0;
    if (kk < ndoc) {
      const int a = (int)(P.doc_sent_off[d0 + kk] - s0), b = (int)(P.doc_sent_off[d0 + kk + 1] - s0);
      const int c = min(a + P.doc_nseg_doc[d0 + kk], b);
      first = kept_before[a];
      cnt = kept_before[b] - first;
      ndseg = kept_before[c] - first;
    }
    const int keep = (kk < ndoc && cnt - ndseg > 0) ? 1 : 0;
    const int incl = wscan_incl(keep, lane);
    if (keep) {
      const int di = nd_docs + incl - 1;
      P.fd_first[d0 + di] = s0 + first;
      P.fd_n[d0 + di] = cnt;
      P.fd_nd[d0 + di] = ndseg;
    }
    nd_docs += lane_get(incl, 63);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  auto len_abs = [&](int64_t slot) -> int { return P.fs_ntok[slot]; };

  WaveRng rng{L, lane, MT_N};
  rng.load(P.mt_states + (int64_t)p * MT_N);
  const int max_doc = P.max_seq >= 512 ? 64 : 32;
  PairRec* out = P.pairs + pb;
  int np = 0;
  int err = PACK_OK;
  for (int dup = 0; dup < P.dup && !err; ++dup) {
    for (int di = 0; di < nd_docs && !err; ++di) {
      const int64_t first = P.fd_first[d0 + di];
      const int nd = P.fd_nd[d0 + di];
      const int nc = P.fd_n[d0 + di] - nd;
      const int64_t cfirst = first + nd;
      const int special = nd ? 3 : 2;
      const int max_num = P.max_seq - special;
      const double sp = rng.random();
      // docstring part (pretrain_codebert.py:375-396)
      int dn = 0, dlo = 0, dhi = 0;
      if (nd && sp < P.short_seq_prob) {
        dn = 1;
        dhi = len_abs(first);
      } else if (nd) {
        int cur;
        // flush at i == nc - 1 (the quirk: the code-segment count) or cur > max_doc
        const int i = find_over([&](int k) { return len_abs(first + k); }, 0, nd, nc - 1, 0, max_doc, lane, &cur);
        if (i >= 0) {
          const int cn = i + 1;
          dn = (cur > max_doc && cn > 1) ? cn - 1 : cn;
          dhi = dn == cn ? cur : cur - len_abs(first + i);
          trunc_seq_wave(rng, L, lane, dlo, dhi, max_doc);
        }
      }
      const int doc_len = dhi - dlo;
      // code part (:400-440): chunks [cs, i], the overflowing segment carried
      int cs = 0, k0 = 0, carried = 0;  // carried: the chunk already holds segment cs (stay)
      int nout = 0;
      while (k0 < nc && !err) {
        const int b0 = doc_len + carried;
        int cur;
        const int i = find_over([&](int k) { return len_abs(cfirst + k); }, k0, nc, nc - 1, b0, max_num, lane, &cur);
        const int cn = i - cs + 1;
        const bool stay = cur > max_num && cn > 1;
        int clo = 0, chi = cur - doc_len;
        const int lim = max_num - doc_len;
        if (lim < 0) { err = PACK_EINDEX; break; }  // del from an empty list: IndexError
        trunc_seq_wave(rng, L, lane, clo, chi, lim);
        if (chi - clo < 1) { err = PACK_EASSERT; break; }
        if (nout == 0 || chi - clo >= 16) {
          if (lane == 0) {
            PairRec r;
            r.fs0 = first; r.n0 = (uint16_t)dn; r.lo0 = (uint16_t)dlo; r.hi0 = (uint16_t)dhi;
            r.fs1 = cfirst + cs; r.n1 = (uint16_t)cn; r.lo1 = (uint16_t)clo; r.hi1 = (uint16_t)chi;
            r.flags = (uint16_t)(special == 3 ? 2 : 0);
            r.num_tokens = (uint16_t)(doc_len + (chi - clo) + special);
            out[np] = r;
          }
          ++np;
          ++nout;
        }
        if (stay) { cs = i; carried = len_abs(cfirst + i); }
        else { cs = i + 1; carried = 0; }
        k0 = i + 1;
      }
    }
  }
  if (lane == 0) P.part_err[p] = err;
  if (err) {
    if (lane == 0) { P.part_npairs[p] = 0; P.part_ntok[p] = 0; }
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  // ---- random.shuffle(partition_pairs) (:476) ------------------------------
  int32_t* gorder = P.order + pb;
  for (int k = lane; k < np; k += 64) gorder[k] = k;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  shuffle_global(rng, np, gorder, P.binned + pb, lane);  // (binned: draw scratch until binning)
  const bool packed = order_packable(np, P.max_seq);
  if (packed) pack_order_nt(gorder, out, np, lane);
  // ---- stable bin partition + token offsets ---------------------------------
  const int nb = P.nbins;
  int32_t* binned = P.binned + pb;
  int64_t* tl = P.tok_local + pb;
  int pos = 0;
  int64_t acc = 0;
  for (int b = 0; b < nb; ++b) {
    int cnt = 0;
    for (int k = 0; k < np; k += 64) {
      const int kk = k + lane;
      int rec = 0, nt = 0;
      bool in = false;
      if (kk < np) {
        const int v = gorder[kk];
        rec = packed ? v & ((1 << PACKED_REC_BITS) - 1) : v;
        nt = packed ? (int)((uint32_t)v >> PACKED_REC_BITS) : (int)out[rec].num_tokens;
        int bb = (nt - 1) / P.bin_size;
        bb = bb > nb - 1 ? nb - 1 : bb;
        in = bb == b;
      }
      const uint64_t m = __ballot(in);
      const int before = __popcll(m & ((1ull << lane) - 1ull));
      const int tinc = wscan_incl(in ? nt : 0, lane);
      if (in) {
        binned[pos + before] = rec;
        tl[pos + before] = acc + tinc - nt;
      }
      pos += __popcll(m);
      cnt += __popcll(m);
      acc += lane_get(tinc, 63);
    }
    if (lane == 0) P.bin_count[p * nb + b] = cnt;
  }
  if (lane == 0) {
    P.part_npairs[p] = np;
    P.part_ntok[p] = acc;
  }
}

hipError_t launch_pack_codebert_wave(const PackParams& P, hipStream_t s) {
  hipLaunchKernelGGL(pack_codebert_wave_kernel, dim3((unsigned)P.n_part), dim3(64), 0, s, P);
  return hipGetLastError();
}

}  // namespace lddl
