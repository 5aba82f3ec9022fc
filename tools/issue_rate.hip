// VALU issue-rate microbenchmark for gfx950 (VERDICT r2 "step one"): how many
// cycles a SIMD spends per wave64 vector instruction of the tokenizer scan's
// instruction mix, at 1..8 waves per SIMD.  Each wave runs ILP independent
// chains of one instruction in an unrolled loop; the SIMD's cycles per
// wave-instruction = (s_memtime cycles of the slowest wave) / (waves per SIMD x
// instructions per wave).  A rate of 2.0 = one wave64 VALU per 2 cycles per
// SIMD (32 lanes per cycle), 4.0 = one per 4 cycles.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/issue_rate tools/issue_rate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                     \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) {                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
      exit(1);                                                       \
    }                                                                \
  } while (0)

constexpr int ITERS = 2048;

enum Op { ADD, XOR, PERM, MUL, ALIGNB, BFE, LSHLOR, DPP, CNDMASK, MIX_SCAN, MIX_LDS, MIX_SALU, NOPS };
static const char* op_name[NOPS] = {"v_add_u32", "v_xor_b32", "v_perm_b32", "v_mul_lo_u32", "v_alignbyte_b32",
                                    "v_bfe_u32", "v_lshl_or_b32", "v_mov_b32_dpp(row_shr:1)", "v_cndmask_b32",
                                    "mix: 6 int VALU + 1 perm + 1 dpp", "mix: 6 VALU + 1 ds_read_b32",
                                    "mix: 6 VALU + 2 SALU"};
// VALU instructions per unrolled step for each op (8 chains)
static const int op_valu[NOPS] = {8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 6, 6};

template <int OP>
__device__ __forceinline__ void step(uint32_t (&v)[8], uint32_t k, uint32_t* lds, uint32_t& s0) {
  if (OP == ADD) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(k));
  } else if (OP == XOR) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[i]) : "v"(k));
  } else if (OP == PERM) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(k), "v"(0x05010400u));
  } else if (OP == MUL) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[i]) : "v"(k));
  } else if (OP == ALIGNB) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(v[i]) : "v"(k));
  } else if (OP == BFE) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_bfe_u32 %0, %0, 3, 9" : "+v"(v[i]));
  } else if (OP == LSHLOR) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(v[i]) : "v"(k));
  } else if (OP == DPP) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(v[i]));
  } else if (OP == CNDMASK) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(k) : "vcc");
  } else if (OP == MIX_SCAN) {
    asm volatile(
        "v_add_u32 %0, %0, %8\n\t"
        "v_xor_b32 %1, %1, %8\n\t"
        "v_perm_b32 %2, %2, %8, %9\n\t"
        "v_and_b32 %3, %3, %8\n\t"
        "v_mov_b32_dpp %4, %4 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_or_b32 %5, %5, %8\n\t"
        "v_lshl_or_b32 %6, %6, 3, %8\n\t"
        "v_bfe_u32 %7, %7, 3, 9"
        : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
        : "v"(k), "v"(0x05010400u));
  } else if (OP == MIX_LDS) {
    uint32_t t;
    asm volatile("ds_read_b32 %0, %1" : "=v"(t) : "v"((uint32_t)(uintptr_t)lds) : "memory");
#pragma unroll
    for (int i = 0; i < 6; ++i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(k));
    asm volatile("s_waitcnt lgkmcnt(0)\n\tv_xor_b32 %0, %0, %1" : "+v"(v[7]) : "v"(t));
  } else if (OP == MIX_SALU) {
#pragma unroll
    for (int i = 0; i < 3; ++i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(k));
    asm volatile("s_add_u32 %0, %0, 7" : "+s"(s0));
#pragma unroll
    for (int i = 3; i < 6; ++i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(k));
    asm volatile("s_xor_b32 %0, %0, 5" : "+s"(s0));
  }
}

template <int OP>
__global__ __launch_bounds__(256) void bench_kernel(uint32_t* out, unsigned long long* cyc, uint32_t seed) {
  __shared__ uint32_t lds[256];
  lds[threadIdx.x] = threadIdx.x * seed;
  __syncthreads();
  uint32_t v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = threadIdx.x * (i + 1) + seed;
  uint32_t s0 = seed;
  const uint32_t k = seed | 1u;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) step<OP>(v, k, lds + (threadIdx.x & 63), s0);
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t acc = s0;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc ^= v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) atomicMax(cyc, (unsigned long long)(t1 - t0));
}

template <int OP>
static double run(int n_cu, int wps, uint32_t* d_out, unsigned long long* d_cyc) {
  // 4 waves per block (one per SIMD); wps blocks per CU -> wps waves per SIMD
  const int blocks = n_cu * wps;
  double best = 1e30;
  for (int rep = 0; rep < 3; ++rep) {
    CHECK(hipMemset(d_cyc, 0, 8));
    hipLaunchKernelGGL(bench_kernel<OP>, dim3(blocks), dim3(256), 0, 0, d_out, d_cyc, 0x9E3779B9u + rep);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    unsigned long long cyc = 0;
    CHECK(hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost));
    const double valu_per_wave = (double)ITERS * 8 * op_valu[OP];
    const double r = (double)cyc / (wps * valu_per_wave);
    if (r < best) best = r;
  }
  return best;
}

template <int OP>
static void row(int n_cu, uint32_t* d_out, unsigned long long* d_cyc) {
  printf("%-36s", op_name[OP]);
  for (int wps : {1, 2, 3, 4, 5, 6, 8}) printf("  %5.2f", run<OP>(n_cu, wps, d_out, d_cyc));
  printf("\n");
  fflush(stdout);
}

int main() {
  int dev = 0, n_cu = 0;
  CHECK(hipSetDevice(dev));
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, dev));
  n_cu = p.multiProcessorCount;
  uint32_t* d_out;
  unsigned long long* d_cyc;
  CHECK(hipMalloc(&d_out, (size_t)n_cu * 8 * 256 * 4));
  CHECK(hipMalloc(&d_cyc, 8));
  printf("%s, %d CUs: shader cycles per wave64 VALU instruction per SIMD (s_memtime of the slowest wave)\n",
         p.gcnArchName, n_cu);
  printf("%-36s  %5s  %5s  %5s  %5s  %5s  %5s  %5s\n", "waves/SIMD ->", "1", "2", "3", "4", "5", "6", "8");
  row<ADD>(n_cu, d_out, d_cyc);
  row<XOR>(n_cu, d_out, d_cyc);
  row<PERM>(n_cu, d_out, d_cyc);
  row<MUL>(n_cu, d_out, d_cyc);
  row<ALIGNB>(n_cu, d_out, d_cyc);
  row<BFE>(n_cu, d_out, d_cyc);
  row<LSHLOR>(n_cu, d_out, d_cyc);
  row<DPP>(n_cu, d_out, d_cyc);
  row<CNDMASK>(n_cu, d_out, d_cyc);
  row<MIX_SCAN>(n_cu, d_out, d_cyc);
  row<MIX_LDS>(n_cu, d_out, d_cyc);
  row<MIX_SALU>(n_cu, d_out, d_cyc);
  CHECK(hipFree(d_out));
  CHECK(hipFree(d_cyc));
  return 0;
}
