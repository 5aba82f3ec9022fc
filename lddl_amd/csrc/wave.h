// Wave64 cross-lane primitives on DPP (gfx950 is GFX9-family: row_shr,
// row_bcast:15/31 and wave_shr:1 are available).  A DPP move is a VALU
// operand modifier, a few cycles; the __shfl_* forms they replace go through
// ds_bpermute at LDS latency, six of them back to back per scan -- the
// dominant latency of the packer's serial pair loop and of the tokenizer's
// per-tile scans.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lddl {

enum : int {
  DPP_ROW_SHR1 = 0x111,
  DPP_ROW_SHR2 = 0x112,
  DPP_ROW_SHR4 = 0x114,
  DPP_ROW_SHR8 = 0x118,
  DPP_WAVE_SHL1 = 0x130,
  DPP_WAVE_SHR1 = 0x138,
  DPP_ROW_BCAST15 = 0x142,
  DPP_ROW_BCAST31 = 0x143,
};

// lanes whose source is out of range (or whose row is masked off) read 0
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW_MASK, 0xF, false);
}

// inclusive prefix sum over the wave (Hillis-Steele in each 16-lane row, then
// the row totals by broadcast)
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t x) {
  x += dpp0<DPP_ROW_SHR1>(x);
  x += dpp0<DPP_ROW_SHR2>(x);
  x += dpp0<DPP_ROW_SHR4>(x);
  x += dpp0<DPP_ROW_SHR8>(x);
  x += dpp0<DPP_ROW_BCAST15, 0xA>(x);
  x += dpp0<DPP_ROW_BCAST31, 0xC>(x);
  return x;
}
__device__ __forceinline__ int wave_incl_add(int x) { return (int)wave_incl_add((uint32_t)x); }

// inclusive max-scan over the wave (unsigned; the out-of-range reads give 0)
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
  x = max(x, dpp0<DPP_ROW_SHR1>(x));
  x = max(x, dpp0<DPP_ROW_SHR2>(x));
  x = max(x, dpp0<DPP_ROW_SHR4>(x));
  x = max(x, dpp0<DPP_ROW_SHR8>(x));
  x = max(x, dpp0<DPP_ROW_BCAST15, 0xA>(x));
  x = max(x, dpp0<DPP_ROW_BCAST31, 0xC>(x));
  return x;
}

// lane l receives lane l-1's value, lane 0 receives 0
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x) { return dpp0<DPP_WAVE_SHR1>(x); }
__device__ __forceinline__ int wave_shr1(int x) { return (int)dpp0<DPP_WAVE_SHR1>((uint32_t)x); }

// lane l receives lane l+1's value, lane 63 receives 0
__device__ __forceinline__ uint32_t wave_shl1(uint32_t x) { return dpp0<DPP_WAVE_SHL1>(x); }

// value of a (wave-uniform) lane
__device__ __forceinline__ uint32_t lane_get(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }
__device__ __forceinline__ int lane_get(int x, int l) { return __builtin_amdgcn_readlane(x, l); }

// this lane's bit of a wave-uniform mask: the mask becomes exec directly
// (s_and_saveexec), where (m >> lane) & 1 costs a 64-bit shift + compare
__device__ __forceinline__ bool lane_in(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
// set bits of a wave-uniform mask below this lane (v_mbcnt)
__device__ __forceinline__ int bits_below(uint64_t m, int base = 0) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)base));
}

// segmented inclusive sum: a lane with h != 0 starts a segment; returns the
// sum from the segment start (or lane 0) to this lane, h becomes "a segment
// start at or before this lane"
__device__ __forceinline__ void wave_seg_incl_add(uint32_t& h, uint32_t& s) {
#define LDDL_SEG_STEP(CTRL, RM)                        \
  {                                                    \
    const uint32_t ph = dpp0<CTRL, RM>(h), ps = dpp0<CTRL, RM>(s); \
    if (!h) {                                          \
      s += ps;                                         \
      h = ph;                                          \
    }                                                  \
  }
  LDDL_SEG_STEP(DPP_ROW_SHR1, 0xF)
  LDDL_SEG_STEP(DPP_ROW_SHR2, 0xF)
  LDDL_SEG_STEP(DPP_ROW_SHR4, 0xF)
  LDDL_SEG_STEP(DPP_ROW_SHR8, 0xF)
  LDDL_SEG_STEP(DPP_ROW_BCAST15, 0xA)
  LDDL_SEG_STEP(DPP_ROW_BCAST31, 0xC)
#undef LDDL_SEG_STEP
}

}  // namespace lddl
