// k_rows_xp.h (microbenchmark A/B, not in the library) — the row pass of N = 16384 with the x transform split 64 x 256 and the
// sub-transforms' exchanges done inside the wave (lane_xchg.h: v_permlane16/32_swap + DPP), so the
// LDS carries only the two transpositions (k_rows_xs: the two transpositions plus two exchanges of
// every 1024-point sub-transform, half of its LDS traffic).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../oceansimulation_amd/csrc/ocean_internal.h"
#include "../../oceansimulation_amd/csrc/device/fft.h"
#include "../../oceansimulation_amd/csrc/device/grid.h"
#include "../../oceansimulation_amd/csrc/device/lane_xchg.h"
#include "../../oceansimulation_amd/csrc/device/memory.h"

namespace oceanfft
{

// x index n = n1 + 64 n2 (n1 < 64, n2 < 256), output k = k2 + 256 k1:
//   X(k2 + 256 k1) = sum_n1 W_64^(n1 k1) [W_N^(n1 k2) Y_n1(k2)],  Y_n1(k2) = sum_n2 x(n1 + 64 n2) W_256^(n2 k2).
// LDS slot of (n1, j) (8-B halves): n1 RS + (j ^ ((n1 >> 2) & 3)), RS = 4 (mod 16). The XOR keeps both
// access shapes conflict-free: 16 lanes writing 16 consecutive n1 at one j (T_in's writes, the loads'
// order) and 16 lanes reading 4 n1 x 4 consecutive j (the wave's own sub-transform order).
template <int LOGN>
struct XpCfg
{
  static constexpr int RS = 260;  // >= 256 slots per n1, = 4 (mod 16)
  static constexpr int TW = ((FftShape<LOGN>::TW_ENTRIES * 8 + 15) / 16) * 16;
  static constexpr int LDS = TW + 64 * RS * 8;
};

__device__ __forceinline__ int xp_slot(int n1, int j) { return n1 * XpCfg<14>::RS + (j ^ ((n1 >> 2) & 3)); }

// One row of both images per 1024-thread workgroup (16 waves), as k_rows_xs; PF of the next image's
// 8 field loads are in flight during the current image's transform.
//   T_in: thread (w, s, p) = (tid >> 6, tid & 3, (tid >> 2) & 15) receives x(n1 + 64 (p + 16 m)),
//         n1 = 4 w + s: four 256-point sub-transforms per wave, one per lane bits 0..1.
//   sub-transform: DFT-16 over m, x W_256^(p m), registers <-> lane bits 2..5 (in the wave), DFT-16:
//         v[m] = Y_n1(p + 16 m); then x W_N^(n1 (p + 16 m)).
//   T_out: thread (k2, q) = ((tid & 15) + 16 (tid >> 6), (tid >> 4) & 3) receives Z_(q + 4 r)(k2), r < 16.
//   outer DFT-64 over n1 = q + 4 r, k1 = a + 16 b: DFT-16 over r, x W_64^(q a), register bits 2..3 <->
//         lane bits 4..5 (permlane swaps), DFT-4 over q: v[c + 4 b] = X(k2 + 256 (c + 4 h + 16 b)),
//         h = (tid >> 4) & 3.
template <int LOGN, int PF>
__global__ __launch_bounds__(1024) void k_rows_xp(FrameParams fp, const float4* __restrict__ spec, float4* __restrict__ maps,
                                                  float* __restrict__ jac, FoamParams foam,
                                                  const float2* __restrict__ tw_glob, int rows, RowSrc rs)
{
  using S = FftShape<LOGN>;
  constexpr int N = S::N, T = S::T, RS = XpCfg<LOGN>::RS;
  static_assert(LOGN == 14 && T == 1024, "one 16-wave row of 16384 per workgroup");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  float2* xs = reinterpret_cast<float2*>(smem + XpCfg<LOGN>::TW);
  load_twiddles<LOGN>(tw, tw_glob);

  const int total = fp.cascades * rows;
  const float dim = (float)N;
  const int lcpr = 31 - __builtin_clz(rs.cpr), cmask = rs.cpr - 1;
  const int wave0 = __builtin_amdgcn_readfirstlane((int)threadIdx.x & ~63);
  float4 fp4[8], nx4[8];
  auto issue = [&](int item, int img, float4* p4, int m0, int m1) __attribute__((always_inline)) {
    const int c = item / rows, yl = item - c * rows;
    const size_t base = ((size_t)c * rows + yl) * rs.lp;
    const int i = opaque((int)threadIdx.x);
#pragma unroll
    for (int m = m0; m < m1; m++)
    {
      const int src = (m * T + sopaque(wave0)) >> lcpr;
      const size_t sb = (size_t)src * rs.src_stride;
      p4[m] = ld4<kStream>(reinterpret_cast<const float4*>((img == 0 ? rs.ab : rs.de) + sb) + base,
                           ((m * T + i) & cmask) * 16);
    }
  };
  int item = blockIdx.x;
  if (PF > 0 && item < total)
    issue(item, 0, fp4, 0, PF);
  for (; item < total; item += gridDim.x)
  {
    const int c = item / rows, yl = item - c * rows;
    const float dk = fp.c[c].dk;
    const float sgy = (yl & 1) ? -1.0f : 1.0f;
    const size_t base = ((size_t)c * rows + yl) * rs.lp;
#pragma unroll
    for (int img = 0; img < 2; img++)
    {
      const int cimg = c * 2 + img;
      const int tid = opaque((int)threadIdx.x), i = tid;
      const float4* sp = spec + (size_t)cimg * N;
      issue(item, img, fp4, PF, 8);
      CPair v[16];  // own lanes in v[m], the -u lanes in v[m + 8] until T_in
#pragma unroll
      for (int m = 0; m < 8; m++)
      {
        const int u = m * T + i;
        const float kx = (float)u * dk;
        const float4 s4 = ld4<0>(sp, (N / 2 - u) * 16);
        const int src = (m * T + sopaque(wave0)) >> lcpr;
        const float2 cc = ld2<0>(reinterpret_cast<const float2*>(rs.c + (size_t)src * rs.src_stride) + base,
                                 (u & cmask) * 8);
        if (img == 0)
        {
          const CPair p = raw_pair(fp4[m]);
          const float Ar = p.re.x, Ai = p.im.x, Br = p.re.y, Bi = p.im.y, Cr = cc.x, Ci = cc.y;
          v[m] = CPair{f2v{(1.0f - kx) * Ar, -Bi - kx * Cr}, f2v{(1.0f - kx) * Ai, Br - kx * Ci}};
          v[m + 8] = CPair{f2v{(1.0f + kx) * Ar + sgy * s4.x, -Bi + kx * Cr + sgy * s4.z},
                           f2v{-(1.0f + kx) * Ai + sgy * s4.y, -Br - kx * Ci + sgy * s4.w}};
        }
        else
        {
          const CPair q = raw_pair(fp4[m]);
          const float Cr = cc.x, Ci = cc.y, Dr = q.re.x, Di = q.im.x, Er = q.re.y, Ei = q.im.y;
          const float kx2 = kx * kx;
          v[m] = CPair{f2v{-(Di - kx2 * Ci), -Er + kx * Di}, f2v{Dr - kx2 * Cr, -Ei - kx * Dr}};
          v[m + 8] = CPair{f2v{-(Di + kx2 * Ci) + sgy * s4.x, -Er - kx * Di + sgy * s4.z},
                           f2v{-Dr - kx2 * Cr + sgy * s4.y, Ei - kx * Dr + sgy * s4.w}};
        }
      }
      if (i == 0)
      {
        const size_t ns = (size_t)rs.nyq_src * rs.src_stride;
        const float kx = -(dim / 2.0f) * dk;
        const float2 cc = ld2<kStream>(reinterpret_cast<const float2*>(rs.c + ns) + base, rs.cpr * 8);
        const float4 t = ld4<kStream>(reinterpret_cast<const float4*>((img == 0 ? rs.ab : rs.de) + ns) + base,
                                      rs.cpr * 16);
        const CPair p = raw_pair(t);
        if (img == 0)
          v[8] = CPair{f2v{(1.0f - kx) * p.re.x, -p.im.y - kx * cc.x}, f2v{(1.0f - kx) * p.im.x, p.re.y - kx * cc.y}};
        else
        {
          const float kx2 = kx * kx;
          v[8] = CPair{f2v{-(p.im.x - kx2 * cc.y), -p.re.y + kx * p.im.x}, f2v{p.re.x - kx2 * cc.x, -p.im.y - kx * p.re.x}};
        }
      }
      if constexpr (PF > 0)
      {
        if (img == 0)
          issue(item, 1, nx4, 0, PF);
        else if (item + (int)gridDim.x < total)
          issue(item + gridDim.x, 0, nx4, 0, PF);
      }
      // ---- T_in: own lanes at n = i + m T, the -u lanes at N - n (thread 0's v[8]: the Nyquist column at N/2)
      const int w = tid >> 6, l = tid & 63, s = l & 3, p = l >> 2;
      const int n1r = 4 * w + s;                           // this thread's sub-transform
      const int rd = n1r * RS + (p ^ (w & 3));             // + 16 m: x(n1r + 64 (p + 16 m))
      const int n1o = i & 63;                              // own lanes: n1 = i mod 64, j = i / 64 + 16 m
      const int wo = xp_slot(n1o, i >> 6);                 // + 16 m
      const int nm = N - i;                                // mirror lanes: n = N - i - m T, j - 16 m
      const int wm = xp_slot(nm & 63, nm >> 6);            // - 16 m (i = 0: n = N, used for m >= 1 only)
      const int wm0 = i == 0 ? xp_slot(0, (N / 2) >> 6) : wm;
      __syncthreads();  // the previous image's T_out reads are done
#pragma unroll
      for (int h = 0; h < 2; h++)
      {
        if (h)
          __syncthreads();
#pragma unroll
        for (int m = 0; m < 8; m++)
        {
          xs[wo + 16 * m] = half_of(v[m], h);
          xs[(m == 0 ? wm0 : wm) - 16 * m] = half_of(v[m + 8], h);
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < 16; m++)
          set_half(v[m], h, xs[rd + 16 * m]);
      }
      // ---- the 256-point sub-transform of n1r, in the wave's registers
      idft16(v);                                       // v[a] = sum_m W_16^(m a) x(p + 16 m)
      apply_stage_twiddles<LOGN>(v, 64 * p, tw);       // x W_256^(p a) = W_N^(64 p a)
      transpose_reg_lanes_2_5(v);                      // lane bits 2..5 <-> register bits: p now indexes a
      idft16(v);                                       // v[b] = Y_n1r(p + 16 b)
      const float2 base_w = twiddle<LOGN>(n1r * p, tw);  // x W_N^(n1r (p + 16 b))
#pragma unroll
      for (int m = 0; m < 16; m++)
        v[m] = cmul(v[m], base_w);
      apply_stage_twiddles<LOGN>(v, 16 * n1r, tw);
      // ---- T_out: thread (k2, q) gathers Z_(q + 4 r)(k2)
      const int q = (tid >> 4) & 3, k2 = (tid & 15) + 16 * w;
#pragma unroll
      for (int h = 0; h < 2; h++)
      {
        if (h)
          __syncthreads();
#pragma unroll
        for (int m = 0; m < 16; m++)
          xs[rd + 16 * m] = half_of(v[m], h);  // (n1r, p + 16 m): T_in's read slots
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; r++)
          set_half(v[r], h, xs[(q + 4 * r) * RS + (k2 ^ (r & 3))]);
      }
      // ---- outer DFT-64 over n1 = q + 4 r
      idft16(v);                                  // v[a] = sum_r W_16^(r a) Z_(q + 4 r)
      apply_stage_twiddles<LOGN>(v, 256 * q, tw); // x W_64^(q a) = W_N^(256 q a)
      swap_reg_lane_bit<2, 4>(v);                 // q -> register bits 2..3, a's bits 2..3 -> lane bits 4..5
      swap_reg_lane_bit<3, 5>(v);
#pragma unroll
      for (int cc4 = 0; cc4 < 4; cc4++)
        idft4(v[cc4], v[cc4 + 4], v[cc4 + 8], v[cc4 + 12]);  // v[c + 4 b] = X(k2 + 256 (c + 4 q + 16 b))
      float4* dst = maps + ((size_t)cimg * rows + yl) * N;
      const int so = (k2 + 1024 * q) * 16;
#pragma unroll
      for (int m = 0; m < 16; m++)
        st4<kStream>(dst + 256 * (m & 3) + 4096 * (m >> 2), so, from_pair(v[m]));
      if (img == 1)
      {
        const float lam = foam.displacement[c];
        float* jb = jac + ((size_t)c * rows + yl) * N;
#pragma unroll
        for (int m = 0; m < 16; m++)
          st1<kStream>(jb + 256 * (m & 3) + 4096 * (m >> 2), (k2 + 1024 * q) * 4,
                       (1.0f + lam * v[m].im.x) * (1.0f + lam * v[m].re.y) - lam * lam * v[m].im.y * v[m].im.y);
      }
#pragma unroll
      for (int m = 0; m < PF; m++)
        fp4[m] = nx4[m];
    }
  }
}

}  // namespace oceanfft
