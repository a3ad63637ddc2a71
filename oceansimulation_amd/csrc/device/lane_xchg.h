// device/lane_xchg.h — intra-wave transpositions of a register index bit with a lane index bit, without
// the LDS: gfx950's v_permlane16_swap / v_permlane32_swap (lane bits 4 and 5) and bank-masked DPP row
// shifts (lane bits 2 and 3). A thread's 16 values v[m] and the wave's 64 lanes form a 16 x 64 array;
// swapping register bit R with lane bit L moves element (.., R = r, .., L = l, ..) to (.., R = l, .., L = r, ..).
// Each swap rewrites half of the values: one permlane instruction per pair of 32-bit registers (it
// writes both), one DPP move per 32-bit register. No LDS traffic, no barrier, no wait on memory.
#pragma once

#include <hip/hip_runtime.h>

#include "device/fft.h"

namespace oceanfft
{

// DPP controls (gfx9 encoding): row_shl:n = 0x100 + n (lane i reads lane i + n of its row of 16),
// row_shr:n = 0x110 + n (lane i reads lane i - n). bank_mask bit b enables lanes 4b .. 4b + 3 of each row.
template <int CTRL, int BANKS>
__device__ __forceinline__ float dpp_update(float old, float src)
{
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), CTRL, 0xF, BANKS, false));
}

// Lane bit LB (2 or 3) <-> the register bit that distinguishes lo (0) from hi (1).
template <int LB>
__device__ __forceinline__ void swap_lane_bit_dpp(float& lo, float& hi)
{
  static_assert(LB == 2 || LB == 3, "row shifts by 4 or 8 within a row of 16");
  constexpr int SH = 1 << LB;
  constexpr int SET = LB == 2 ? 0xA : 0xC, CLEAR = LB == 2 ? 0x5 : 0x3;  // banks whose lanes have bit LB set / clear
  const float nlo = dpp_update<0x110 + SH, SET>(lo, hi);    // lanes with bit LB: hi of lane - SH
  const float nhi = dpp_update<0x100 + SH, CLEAR>(hi, lo);  // lanes without it: lo of lane + SH
  lo = nlo;
  hi = nhi;
}

// Lane bit 4 (permlane16_swap: odd rows of lo <-> even rows of hi) or 5 (permlane32_swap: the upper
// half of lo <-> the lower half of hi).
template <int LB>
__device__ __forceinline__ void swap_lane_bit_perm(float& lo, float& hi)
{
  static_assert(LB == 4 || LB == 5, "permlane swaps exchange rows (bit 4) or halves (bit 5)");
  unsigned a = __float_as_uint(lo), b = __float_as_uint(hi);
  if constexpr (LB == 4)
  {
    const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    a = r[0];
    b = r[1];
  }
  else
  {
    const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    a = r[0];
    b = r[1];
  }
  lo = __uint_as_float(a);
  hi = __uint_as_float(b);
}

template <int LB>
__device__ __forceinline__ void swap_lane_bit_f(float& lo, float& hi)
{
  if constexpr (LB >= 4)
    swap_lane_bit_perm<LB>(lo, hi);
  else
    swap_lane_bit_dpp<LB>(lo, hi);
}

template <int LB>
__device__ __forceinline__ void swap_lane_bit(CPair& lo, CPair& hi)
{
  // split-plane components (vector elements cannot bind to references)
  float a[4] = {lo.re.x, lo.re.y, lo.im.x, lo.im.y}, b[4] = {hi.re.x, hi.re.y, hi.im.x, hi.im.y};
#pragma unroll
  for (int k = 0; k < 4; k++)
    swap_lane_bit_f<LB>(a[k], b[k]);
  lo = CPair{f2v{a[0], a[1]}, f2v{a[2], a[3]}};
  hi = CPair{f2v{b[0], b[1]}, f2v{b[2], b[3]}};
}

// Register bit RB of v[0..15] <-> lane bit LB.
template <int RB, int LB>
__device__ __forceinline__ void swap_reg_lane_bit(CPair* v)
{
#pragma unroll
  for (int m = 0; m < 16; m++)
    if (!(m & (1 << RB)))
      swap_lane_bit<LB>(v[m], v[m | (1 << RB)]);
}

// The 4 x 4 transposition register bits 0..3 <-> lane bits 2..5 (the four swaps commute).
__device__ __forceinline__ void transpose_reg_lanes_2_5(CPair* v)
{
  swap_reg_lane_bit<0, 2>(v);
  swap_reg_lane_bit<1, 3>(v);
  swap_reg_lane_bit<2, 4>(v);
  swap_reg_lane_bit<3, 5>(v);
}

}  // namespace oceanfft
