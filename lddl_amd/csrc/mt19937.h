// CPython-exact MT19937 (Modules/_randommodule.c + Lib/random.py) for one
// lane, state in global memory.
//
// The reference draws every packing decision from the stdlib `random`
// module (lddl/dask/bert/pretrain.py:173,264-265,286,295,304,313,401), so
// bit-exact pairs need bit-exact draws:
//   seed(n)          init_by_array(|n| as little-endian 32-bit words)
//   random()         (a>>5, b>>6) -> (a*2^26 + b) / 2^53
//   getrandbits(k)   genrand_uint32() >> (32-k)            (k <= 32)
//   _randbelow(n)    k = n.bit_length(); redraw while r >= n
//   randint(a, b)    a + _randbelow(b - a + 1)
//   shuffle(x)       for i = n-1..1: j = _randbelow(i+1); swap
//
// Layout: the 624-word state of lane l of group g (64 partitions per group)
// is 156 uint4 chunks at mt[(g*156 + c)*64 + l]: 16 B per lane, lanes
// interleaved, so a wave twisting in step touches 1 KiB contiguous per chunk.
#pragma once
#include "common.h"

namespace lddl {

struct MTLane {
  uint4* S;        // &mt[(g*156)*64 + l]; chunk c at S[c*64]
  uint4 buf;       // current chunk (cached)
  int idx;         // 0..624

  __device__ __forceinline__ uint4& chunk(int c) const { return S[(size_t)c * 64]; }

  __device__ void seed(uint64_t n) {
    // init_genrand(19650218) then init_by_array(key)
    uint32_t key[2] = {(uint32_t)n, (uint32_t)(n >> 32)};
    const int klen = (n >> 32) ? 2 : 1;
    uint32_t mt[4];
    // streaming init: keep the whole array in global memory, chunk by chunk
    // pass 0: init_genrand
    uint32_t prev = 19650218u;
    for (int c = 0; c < 156; ++c) {
      for (int k = 0; k < 4; ++k) {
        const int i = c * 4 + k;
        if (i == 0) mt[k] = prev;
        else mt[k] = prev = 1812433253u * (prev ^ (prev >> 30)) + (uint32_t)i;
      }
      chunk(c) = make_uint4(mt[0], mt[1], mt[2], mt[3]);
    }
    auto get = [&](int i) -> uint32_t {
      const uint4 v = chunk(i >> 2);
      const int k = i & 3;
      return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
    };
    auto set = [&](int i, uint32_t x) {
      uint4& v = chunk(i >> 2);
      const int k = i & 3;
      if (k == 0) v.x = x; else if (k == 1) v.y = x; else if (k == 2) v.z = x; else v.w = x;
    };
    int i = 1, j = 0;
    uint32_t last = get(0);
    for (int k = MT_N > klen ? MT_N : klen; k; --k) {
      const uint32_t v = (get(i) ^ ((last ^ (last >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
      set(i, v);
      last = v;
      ++i; ++j;
      if (i >= MT_N) { set(0, get(MT_N - 1)); last = get(0); i = 1; }
      if (j >= klen) j = 0;
    }
    for (int k = MT_N - 1; k; --k) {
      const uint32_t v = (get(i) ^ ((last ^ (last >> 30)) * 1566083941u)) - (uint32_t)i;
      set(i, v);
      last = v;
      ++i;
      if (i >= MT_N) { set(0, get(MT_N - 1)); last = get(0); i = 1; }
    }
    set(0, 0x80000000u);
    idx = MT_N;
  }

  __device__ __forceinline__ static uint32_t mix(uint32_t a, uint32_t b, uint32_t m) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }

  // In-place twist in chunk order.  Reading a chunk with a higher index
  // yields the old word, a lower index the new one -- exactly the sequential
  // generator's dependences (mt[kk+1] old, mt[kk+M] old for kk < N-M and
  // new after, mt[0] new for kk = N-1).
  __device__ void twist() {
    uint4 cur = chunk(0);
    uint4 ma = chunk(99);
    for (int c = 0; c < 156; ++c) {
      const int cn = c + 1 == 156 ? 0 : c + 1;
      const int cb = c + 100 >= 156 ? c + 100 - 156 : c + 100;
      const uint4 nxt = chunk(cn);  // c = 155: chunk 0, already new
      const uint4 mb = chunk(cb);
      uint4 o;
      o.x = mix(cur.x, cur.y, ma.y);
      o.y = mix(cur.y, cur.z, ma.z);
      o.z = mix(cur.z, cur.w, ma.w);
      o.w = mix(cur.w, nxt.x, mb.x);
      chunk(c) = o;
      cur = (cn == 0) ? o : nxt;  // not used after c = 155
      ma = mb;
    }
    idx = 0;
  }

  __device__ __forceinline__ uint32_t next() {
    if (idx >= MT_N) twist();
    if ((idx & 3) == 0) buf = chunk(idx >> 2);
    const int k = idx & 3;
    uint32_t y = k == 0 ? buf.x : k == 1 ? buf.y : k == 2 ? buf.z : buf.w;
    ++idx;
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }

  __device__ __forceinline__ double random() {
    const uint32_t a = next() >> 5, b = next() >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
  }

  // _randbelow(n), 1 <= n < 2^32
  __device__ __forceinline__ uint32_t randbelow(uint32_t n) {
    const int k = 32 - __clz(n);
    uint32_t r = next() >> (32 - k);
    while (r >= n) r = next() >> (32 - k);
    return r;
  }

  __device__ __forceinline__ int64_t randint(int64_t a, int64_t b) {
    return a + (int64_t)randbelow((uint32_t)(b - a + 1));
  }
};

}  // namespace lddl
