// FETCH_SIZE / WRITE_SIZE calibration for the access patterns of the
// tokenizer (tools/gpu_calib.sh): reads a known byte count (1 GiB) with
//   mode 0: one 16-B load per lane, contiguous across the wave
//   mode 1: two 16-B non-temporal loads per lane at a 32-B lane stride
//           (tok4's window load, tokenize_stream.hip)
// and writes 2-B ids in ~460-B runs at 1 KiB stride (mode 2, tok4's output);
// random vocab-bucket probes over a 4 GiB table (past the 256 MiB MALL, so
// every probe is a miss at the memory side): 32 B per lane (two 16-B loads of
// one 64-B bucket: the scan's first probe) and 64 B per lane (the whole
// bucket: WordPiece's probe), 2^24 probes each.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ void rd16(const u32x4* p, size_t n, unsigned* sink) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const u32x4 a = p[i];
    acc ^= a.x ^ a.y ^ a.z ^ a.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void rd32nt(const u32x4* p, size_t n32, unsigned* sink) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n32; i += (size_t)gridDim.x * blockDim.x) {
    const u32x4 a = __builtin_nontemporal_load(p + 2 * i), b = __builtin_nontemporal_load(p + 2 * i + 1);
    acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// one wave per 1 KiB tile writes 230 u16 ids starting at a ragged offset
__global__ void wr_runs(unsigned short* out, size_t n_tiles) {
  const int lane = threadIdx.x & 63;
  const size_t t = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  if (t >= n_tiles) return;
  const size_t base = t * 230 + (t * 7) % 3;
  for (int k = lane; k < 230; k += 64) out[base + k] = (unsigned short)(k + t);
}

__device__ __forceinline__ unsigned hmix(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
// NB 16-B loads per lane from a random 64-B bucket of nbk buckets
template <int NB>
__global__ void rnd_probe(const u32x4* t, unsigned nbk_mask, size_t n, unsigned* sink) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const u32x4* b = t + 4 * (size_t)(hmix((unsigned)i * 2654435761u + 12345u) & nbk_mask);
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const u32x4 a = b[k];
      acc ^= a.x ^ a.y ^ a.z ^ a.w;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  void* p;
  unsigned* sink;
  if (hipMalloc(&p, bytes + 4096) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
  hipMemset(p, 1, bytes);
  hipDeviceSynchronize();
  rd16<<<4096, 256>>>((const u32x4*)p, bytes / 16, sink);
  rd32nt<<<4096, 256>>>((const u32x4*)p, bytes / 32, sink);
  const size_t n_tiles = bytes / 1024;  // ids region: 230 * 2 B per tile fits
  wr_runs<<<(unsigned)((n_tiles * 64 + 255) / 256), 256>>>((unsigned short*)p, n_tiles);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("read bytes per kernel %zu; wr_runs algorithmic bytes %zu\n", bytes, n_tiles * 230 * 2);
  const size_t tbytes = (size_t)4 << 30, nprobe = (size_t)1 << 24;
  void* tb;
  if (hipMalloc(&tb, tbytes) != hipSuccess) return 3;
  hipMemset(tb, 3, tbytes);
  hipDeviceSynchronize();
  const unsigned mask = (unsigned)(tbytes / 64 - 1);
  rnd_probe<2><<<4096, 256>>>((const u32x4*)tb, mask, nprobe, sink);
  rnd_probe<4><<<4096, 256>>>((const u32x4*)tb, mask, nprobe, sink);
  if (hipDeviceSynchronize() != hipSuccess) return 4;
  printf("rnd_probe: %zu probes of 32 B (%zu B) and of 64 B (%zu B) over a %zu-B table\n", nprobe, nprobe * 32,
         nprobe * 64, tbytes);
  return 0;
}
