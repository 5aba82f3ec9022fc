// Measurement probe (not product code): how fast is the core of a
// byte-parallel tokenizer design -- one thread per 32-byte chunk, no wave
// cooperation, no per-unit chain across lanes -- on the real vocab table?
// Each thread finds the word starts in its chunk (ASCII letters / digits;
// bytes >= 0x80 count as word bytes and send the word to a slow path), takes
// each word's length from its own and the next chunk's word masks, gathers
// and lowercases up to 24 key bytes, hashes them and probes slot 0 of the
// home bucket exactly as tok5's scan does (common.h vhash / slot layout,
// tok_tables.h build_vocab_tables).  No sentences, entries, records or
// normalisation exceptions: an optimistic bound on that design's fast path,
// to hold against the scan's 3.4 ms per GB.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lddl_amd/csrc -o ab/bytepar_probe tools/bytepar_probe.hip
//   ab/bytepar_probe VOCAB CORPUS [REPS]
// modes: 0 word starts and lengths only; 1 + key gather, hash and probe;
// 2 + the found ids stored (16 u16 per thread).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "common.h"
#include "tok_tables.h"

using namespace lddl;

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

__device__ __forceinline__ uint32_t word_bits(uint32_t x) {  // byte j word char -> bit j (of 4)
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t c = (x >> (8 * j)) & 0xFFu, l = c | 0x20u;
    const bool w = c >= 0x80u || (l - 'a') < 26u || (c - '0') < 10u;
    m |= (w ? 1u : 0u) << j;
  }
  return m;
}
__device__ __forceinline__ uint32_t lower4(uint32_t x) {  // ASCII A-Z -> a-z (bytes < 0x80)
  const uint32_t h = x & 0x7F7F7F7Fu;
  const uint32_t ge = h + 0x3F3F3F3Fu;  // >= 'A' sets bit 7 (0x80 - 'A' = 0x3F)
  const uint32_t gt = h + 0x25252525u;  // > 'Z' sets bit 7 (0x80 - 'Z' - 1 = 0x25)
  return x | (((ge & ~gt & ~x) & 0x80808080u) >> 2);
}
__device__ __forceinline__ uint32_t keep(uint32_t c, int rem) {
  return rem >= 4 ? c : rem <= 0 ? 0u : (c & ((1u << (8 * rem)) - 1u));
}

template <int MODE>
__global__ __launch_bounds__(256) void probe_kernel(const uint8_t* __restrict__ bytes, int64_t n,
                                                    const uint4* __restrict__ vt, uint32_t vmask,
                                                    uint16_t* __restrict__ out, unsigned long long* cnt) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t p0 = t * 32;
  uint32_t m = 0, words = 0, hits = 0, slow = 0, lng = 0;
  uint32_t prevw = 0;
  if (p0 < n) {
    const uint4 a = reinterpret_cast<const uint4*>(bytes + p0)[0], b = reinterpret_cast<const uint4*>(bytes + p0)[1];
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) m |= word_bits(w[k]) << (4 * k);
    const int64_t lim = n - p0;  // bytes past the corpus end are not word bytes
    if (lim < 32) m &= (1u << lim) - 1u;
    prevw = p0 > 0 ? (word_bits(bytes[p0 - 1]) & 1u) : 0u;
  }
  // the next chunk's mask from the next lane; the wave's last lane computes its own
  uint32_t mn = __shfl_down(m, 1);
  if ((threadIdx.x & 63) == 63 && p0 + 32 < n) {
    const uint4 a = reinterpret_cast<const uint4*>(bytes + p0 + 32)[0], b = reinterpret_cast<const uint4*>(bytes + p0 + 32)[1];
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    mn = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) mn |= word_bits(w[k]) << (4 * k);
    const int64_t lim = n - p0 - 32;
    if (lim < 32) mn &= (1u << lim) - 1u;
  } else if ((threadIdx.x & 63) == 63) {
    mn = 0;
  }
  const uint64_t M = (uint64_t)m | ((uint64_t)mn << 32);
  uint32_t starts = m & ~((m << 1) | prevw);
  int k_out = 0;
  while (starts) {
    const int i = __ffs(starts) - 1;
    starts &= starts - 1;
    const uint64_t run = ~(M >> i);
    const int len = run ? __builtin_ctzll(run) : 64;
    ++words;
    if (MODE == 0) continue;
    if (len > 24) {
      ++lng;
      continue;
    }
    const int64_t p = p0 + i;
    const uint32_t* d = reinterpret_cast<const uint32_t*>(bytes + (p & ~(int64_t)3));
    const uint32_t sh = (uint32_t)(p & 3);
    uint32_t x[8];
#pragma unroll
    for (int q = 0; q < 7; ++q) x[q] = d[q];
    uint32_t k6[6];
    uint32_t hi = 0;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      k6[q] = keep(__builtin_amdgcn_alignbyte(x[q + 1], x[q], sh), len - 4 * q);
      hi |= k6[q];
      k6[q] = lower4(k6[q]);
    }
    if (hi & 0x80808080u) {  // non-ASCII: the design's slow path
      ++slow;
      continue;
    }
    const uint32_t h = vfinal(vmix(vmix(vmix(VSEED, k6[0]), k6[1]), k6[2]), (uint32_t)len, 0u);
    const uint4* bk = vt + 4 * (h & vmask);
    const uint4 fa = bk[0], fb = bk[1];
    const uint32_t diff = ((fb.z & 0xFFFF0000u) ^ (((uint32_t)len << 16) | 0x80000000u)) | (fa.x ^ k6[0]) |
                          (fa.y ^ k6[1]) | (fa.z ^ k6[2]) | (fa.w ^ k6[3]) | (fb.x ^ k6[4]) | (fb.y ^ k6[5]);
    const bool hit = diff == 0u;
    hits += hit ? 1u : 0u;
    if (MODE == 2 && k_out < 16) out[t * 16 + k_out++] = hit ? (uint16_t)(fb.z & 0xFFFFu) : (uint16_t)0xFFFFu;
  }
  // one atomic per wave per counter
  uint32_t v[4] = {words, hits, slow, lng};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    uint32_t s = v[c];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(&cnt[c], (unsigned long long)s);
  }
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: bytepar_probe VOCAB CORPUS [REPS]\n");
    return 2;
  }
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  VocabTables V;
  std::string err;
  if (build_vocab_tables(argv[1], V, err, false) != 0) {
    fprintf(stderr, "vocab: %s\n", err.c_str());
    return 1;
  }
  FILE* f = fopen(argv[2], "rb");
  if (!f) {
    perror(argv[2]);
    return 1;
  }
  fseek(f, 0, SEEK_END);
  const int64_t n = ftell(f);
  fseek(f, 0, SEEK_SET);
  std::vector<uint8_t> h((size_t)n + 256, 0);  // (zero pad: the last chunks' 16-B and key over-reads)
  if (fread(h.data(), 1, (size_t)n, f) != (size_t)n) return 1;
  fclose(f);
  uint8_t* d_bytes;
  uint4* d_vt;
  uint16_t* d_out;
  unsigned long long* d_cnt;
  const int64_t nthr = (n + 31) / 32;
  CK(hipMalloc(&d_bytes, h.size()));
  CK(hipMemcpy(d_bytes, h.data(), h.size(), hipMemcpyHostToDevice));
  CK(hipMalloc(&d_vt, V.vt.size() * 4));
  CK(hipMemcpy(d_vt, V.vt.data(), V.vt.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&d_out, (size_t)nthr * 16 * 2));
  CK(hipMalloc(&d_cnt, 4 * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned grid = (unsigned)((nthr + 255) / 256);
  printf("corpus %.3f GB, %lld threads, vocab table %.1f MB\n", n / 1e9, (long long)nthr, V.vt.size() * 4 / 1e6);
  for (int mode = 0; mode < 3; ++mode) {
    float best = 1e30f;
    unsigned long long c[4] = {0, 0, 0, 0};
    for (int r = 0; r < reps; ++r) {
      CK(hipMemset(d_cnt, 0, 32));
      CK(hipEventRecord(e0, 0));
      if (mode == 0) hipLaunchKernelGGL(probe_kernel<0>, dim3(grid), dim3(256), 0, 0, d_bytes, n, d_vt, V.vt_mask, d_out, d_cnt);
      else if (mode == 1) hipLaunchKernelGGL(probe_kernel<1>, dim3(grid), dim3(256), 0, 0, d_bytes, n, d_vt, V.vt_mask, d_out, d_cnt);
      else hipLaunchKernelGGL(probe_kernel<2>, dim3(grid), dim3(256), 0, 0, d_bytes, n, d_vt, V.vt_mask, d_out, d_cnt);
      CK(hipGetLastError());
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
      CK(hipMemcpy(c, d_cnt, 32, hipMemcpyDeviceToHost));
    }
    printf("mode %d: %.3f ms = %.3f ms per GB; words %llu (%.3f per byte), whole-word hits %llu (%.1f %%), "
           "non-ASCII %llu, > 24 B %llu\n",
           mode, best, best / (n / 1e9), c[0], (double)c[0] / n, c[1], c[0] ? 100.0 * c[1] / c[0] : 0.0, c[2], c[3]);
  }
  return 0;
}
