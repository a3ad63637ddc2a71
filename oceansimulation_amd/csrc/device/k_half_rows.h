// device/k_half_rows.h — the half-spectrum row pass: rebuild the reference's four packed lanes
// from the kept half (Hermitian symmetry + the Nyquist-row term), x iFFT, maps and Jacobian
// (resources/spectrum.compute:246-259).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ocean_internal.h"
#include "device/evolve.h"
#include "device/fft.h"
#include "device/grid.h"
#include "device/memory.h"
#include "device/spectrum.h"
#include "device/k_half_cols.h"

namespace oceanfft
{

// Pass 2: RPW rows of one image. Element m of the x transform is column x = ((m + 8) & 15) T + i,
// u = x - N/2: m < 8 -> u = m T + i >= 0 (stored column u), m >= 8 -> u < 0. Every thread loads
// only its 8 direct elements (and thread 0 the Nyquist column for m = 8) and computes the lanes
// both at u (its own) and at -u, adding there the Nyquist-row term (-1)^y S(-u); the -u lanes go
// through LDS to the thread that holds -u: element 15 - m of thread T - i (thread 0: element
// 16 - m of itself). Each stored value is read once from HBM. Then the x-iFFT, maps + Jacobian.
// ABL (tools/microbench timing ablations, results wrong by construction): 1 = no HBM loads,
// 2 = no x transform, 3 = no mirror exchange through LDS.
// RPW_ = 2 (default): 512-thread workgroups, two per CU, so one workgroup's loads overlap the
// other's transform (the LDS mirror exchange adds a barrier the 1024-thread, one-per-CU shape cannot
// hide: 1.92 -> 1.69 ms at 8 x 4096^2, tools/microbench/genbench).
// BOTH: one item = both images of its rows (image 0, then image 1), so C is loaded once and kept
// in VGPRs (16) for image 1 instead of being fetched again by a second item.
// RM (row-major fields; RowSrc): element u in [0, N/2) of local row y of cascade c lies in source
// block u / cpr at ((c rows + y) lp + u % cpr), the Nyquist column u = -N/2 in block nyq_src at column
// cpr; the pass covers `rows` rows (a slab's w). The strip-dealt path (after k_half_to_rows) is one
// block [c][rows][N/2 + B]; the four-step path reads the exchange blocks of every source rank directly.
// cpr is a multiple of the 32 consecutive u one wave loads, so the block index is wave-uniform.
// RG / RGC (whole grids): the field layout pass 1 wrote (half_group_offset).
// FB: the field strips' width (half_group_offset); GRP: consecutive items run together on one XCD
// (2: pairs, xcd_pair_slot; 4: FB = 2 with RGC = 8, where four items share each gc line).
// XS (RPW = 1, N = 16 T, T = 1024: one row per 16-wave workgroup): the x transform in four steps
// so that most of it runs between workgroup barriers instead of across them. With n = n1 + 16 n2
// and k = k2 + T k1: a transposition through LDS (T_in, which also does the mirror exchange's job)
// gives wave n1 the T inputs x(n1 + 16 n2); each wave runs its T-point sub-transform (fft_run<LOGN -
// 4>, 64 lanes x 16 points) in its own LDS region, ordered by the LDS's in-order execution of one
// wave's instructions instead of barriers; twiddles W_N^(n1 k2); a second transposition (T_out)
// gives thread k2 the 16 values over n1, and a 16-point DFT in registers leaves X(k2 + T k1) in the
// plain path's layout (coalesced stores). Barriers per image: 7 instead of 14 (mirror 2 + three
// exchanges of two halves x 2 + 1). rm16bench priced the barriers of the 16384 pass at ~1 ms of
// 3.8. tw2_glob: the T-point table (appended for 8192/16384 by ocean_fft_create).
template <int LOGN>
struct XsCfg
{
  static constexpr int L2 = LOGN - 4;
  // region of one n1 (slots of 8 B): holds a sub-transform's padded exchange (PADDED + 4), and
  // RS = 1 mod 16 spreads T_in's 16-lane writes (16 regions at once) over all 32 banks
  static constexpr int RS = ((FftShape<L2>::PADDED + 4 + 14) / 16) * 16 + 1;
  static constexpr int TW1 = ((FftShape<LOGN>::TW_ENTRIES * 8 + 15) / 16) * 16;
  static constexpr int TW2 = ((FftShape<L2>::TW_ENTRIES * 8 + 15) / 16) * 16;
  static constexpr int LDS = TW1 + TW2 + 16 * RS * 8;
};

template <int LOGN, int LA = kStream, int SA = kStream, int ABL = 0, int RPW_ = 2, bool BOTH = false, bool RM = false,
          int RG = 1, int RGC = 1, int FB = 4, int GRP = 2, bool IL = true, bool XS = false>
__global__ __launch_bounds__(FftShape<LOGN>::T * RPW_) void k_rows_half(
    FrameParams fp, const float4* __restrict__ gab, const float4* __restrict__ gde, const float2* __restrict__ gc,
    const float4* __restrict__ spec, float4* __restrict__ maps, float* __restrict__ jac, FoamParams foam,
    const float2* __restrict__ tw_glob, int rows, RowSrc rs, const float2* __restrict__ tw2_glob)
{
  using S = FftShape<LOGN>;
  using K = ColFirstCfg<LOGN>;
  using HC = HalfCfg<LOGN>;
  constexpr int N = S::N, T = S::T, B = K::B, RPW = RPW_, STRIPS = HC::STRIPS, WG = T * RPW;
  static_assert(WG * 8 * 16 <= lds_row_slots<LOGN>(RPW) * 8, "mirror exchange fits the transform's LDS");
  static_assert(!XS || (RPW == 1 && T == 1024), "XS: one 16-wave row per workgroup");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  float2* tw2 = reinterpret_cast<float2*>(smem + XsCfg<LOGN>::TW1);
  void* xch = smem + (XS ? XsCfg<LOGN>::TW1 + XsCfg<LOGN>::TW2 : ((S::TW_ENTRIES * 8 + 15) / 16) * 16);
  CPair* mir = reinterpret_cast<CPair*>(xch);  // [m < 8][thread]: lanes at -u for the partner
  if constexpr (XS)
  {
    for (int e = threadIdx.x; e < FftShape<XsCfg<LOGN>::L2>::TW_ENTRIES; e += blockDim.x)
      tw2[e] = tw2_glob[e];
  }
  load_twiddles<LOGN>(tw, tw_glob);

  const int blocks = (RM ? rows : N) / RPW;
  const int b0 = threadIdx.x % B, r0 = (threadIdx.x / B) % RPW, ihi0 = threadIdx.x / (B * RPW);
  // After the first exchange: RPW = 2 interleaves the two rows (lanes: row fastest) and their LDS
  // regions (CI = 2, slot = 2 pa + row), so a wave's reads of 32 consecutive positions never straddle
  // a pad slot: conflict-free exchanges at 4096 (the row layout cost one extra cycle per 32-lane read
  // group, 262 K LDS cycles per CU per frame = SQ_LDS_BANK_CONFLICT; tools/lds_banks.py models both).
  // (A/B, halfbench rows: 1.449 -> 1.417 ms at 8 x 4096^2, 0.341 -> 0.335 at 2048; at 1024 the row
  // layout stays: 0.079 vs 0.083 ms). IL = false: the row layout.
  constexpr int CI = (IL && RPW == 2 && T >= 128) ? 2 : 0;
  const int i20 = CI ? (threadIdx.x / RPW) % T : threadIdx.x % T, r20 = CI ? threadIdx.x % RPW : threadIdx.x / T;
  const int total = fp.cascades * (BOTH ? 1 : 2) * blocks;
  const float dim = (float)N;
  // RPW = 2: C's row pairs are 64-B halves of 128-B lines; items 2p, 2p+1 (the same line) run
  // together on one XCD so the line is fetched once
  // (RPW = 1 with GRP = 4, an A/B: the 4 rows of a gc line on one XCD)
  for (int item = RPW != 2 && GRP != 4 ? blockIdx.x : GRP == 4 ? xcd_group_slot<4>(blockIdx.x, gridDim.x)
                                                                : xcd_pair_slot(blockIdx.x, gridDim.x);
       item < total; item += gridDim.x)
  {
    const int cimg0 = item / blocks, y0 = (item - cimg0 * blocks) * RPW;
    float2 ckeep[8];  // BOTH: image 0's C loads, reused by image 1
    float2 cnyq;
#pragma unroll
    for (int pass = 0; pass < (BOTH ? 2 : 1); pass++)
    {
    const int cimg = BOTH ? cimg0 * 2 + pass : cimg0;
    const int b = opaque(b0), ihi = opaque(ihi0), r = RPW == 1 ? 0 : opaque(r0);
    const int i = ihi * B + b;
    const int c = cimg >> 1, img = BOTH ? pass : (cimg & 1);
    const float dk = fp.c[c].dk;
    // RM: the item's first row in every source block (texels); element (r, u) at r lp + u % cpr
    const size_t base = RM ? ((size_t)c * rows + y0) * rs.lp : (size_t)c * STRIPS * N * B;
    const int y = y0 + r;
    const float sgy = (y & 1) ? -1.0f : 1.0f;  // (-1)^q of the Nyquist-row term
    const float4* sp = spec + (size_t)cimg * N;
    const int tid = opaque((int)threadIdx.x);
    CPair v[16];  // XS: own lanes in v[m], the -u lanes in v[m + 8] until the transposition
#pragma unroll
    for (int m = 0; m < 8; m++)
    {
      const int u = m * T + i;               // >= 0, column x = N/2 + u
      // source block (wave-uniform; cpr a power of two, launch_rm_rows): a shift, not a division
      const int src = RM ? __builtin_amdgcn_readfirstlane(u >> (31 - __builtin_clz(rs.cpr))) : 0;
      const int off = RM ? r * rs.lp + (u & (rs.cpr - 1)) : half_group_offset<LOGN, RG, FB>(y, u / FB, u % FB);
      const int offc = RM ? off : half_group_offset<LOGN, RGC, FB>(y, u / FB, u % FB);
      const float4* fab = RM ? reinterpret_cast<const float4*>(rs.ab + src * rs.src_stride) + base : gab + base;
      const float4* fde = RM ? reinterpret_cast<const float4*>(rs.de + src * rs.src_stride) + base : gde + base;
      const float2* fc = RM ? reinterpret_cast<const float2*>(rs.c + src * rs.src_stride) + base : gc + base;
      const float kx = (float)u * dk;        // ((float)x - N/2) dk, x - N/2 exact
      const float4 s4 = ld4<0>(sp, (N / 2 - u) * 16);  // the -u column's Nyquist-row term (x = N/2 - u)
      CPair own, neg;
      if (ABL == 1)
      {
        own = CPair{f2v{kx, s4.x}, f2v{(float)off, sgy}};
        neg = CPair{f2v{s4.y, kx}, f2v{sgy, (float)u}};
      }
      else if (img == 0)
      {
        const CPair p = raw_pair(ld4<LA>(fab, off * 16));  // (A, B)
        const float2 cc = ld2<LA>(fc, offc * 8);             // C
        if (BOTH)
          ckeep[m] = cc;
        const float Ar = p.re.x, Ai = p.im.x, Br = p.re.y, Bi = p.im.y, Cr = cc.x, Ci = cc.y;
        // at u: lane0 = (1 - kx) A, lane1 = i B - kx C
        own = CPair{f2v{(1.0f - kx) * Ar, -Bi - kx * Cr}, f2v{(1.0f - kx) * Ai, Br - kx * Ci}};
        // at -u (kx -> -kx, A -> conj A, B -> -conj B, C -> conj C): lane0 = (1 + kx) conj A,
        // lane1 = i (-conj B) + kx conj C
        neg = CPair{f2v{(1.0f + kx) * Ar + sgy * s4.x, -Bi + kx * Cr + sgy * s4.z},
                    f2v{-(1.0f + kx) * Ai + sgy * s4.y, -Br - kx * Ci + sgy * s4.w}};
      }
      else
      {
        const CPair q = raw_pair(ld4<LA>(fde, off * 16));  // (D, E)
        const float2 cc = BOTH ? ckeep[m] : ld2<LA>(fc, offc * 8);  // C
        const float Cr = cc.x, Ci = cc.y, Dr = q.re.x, Di = q.im.x, Er = q.re.y, Ei = q.im.y;
        const float kx2 = kx * kx;
        // at u: lane2 = i (D - kx^2 C), lane3 = -E - i kx D
        own = CPair{f2v{-(Di - kx2 * Ci), -Er + kx * Di}, f2v{Dr - kx2 * Cr, -Ei - kx * Dr}};
        // at -u (D -> -conj D, C -> conj C, E -> conj E, kx -> -kx): lane2 = i (-conj D - kx^2 conj C),
        // lane3 = -conj E + i kx (-conj D)
        neg = CPair{f2v{-(Di + kx2 * Ci) + sgy * s4.x, -Er - kx * Di + sgy * s4.z},
                    f2v{-Dr - kx2 * Cr + sgy * s4.y, Ei - kx * Dr + sgy * s4.w}};
      }
      v[m] = own;
      if constexpr (ABL == 3 || XS)
        v[m + 8] = neg;
      else
        mir[m * WG + tid] = neg;
    }
    if constexpr (ABL != 3 && !XS)
      __syncthreads();
    // own elements m >= 8 (u < 0): from the partner's mirror slots; thread 0's m = 8 is the Nyquist
    // column (u = -N/2), read directly
    const int tp = i == 0 ? tid : tid + (((T - i) / B - ihi) * B * RPW) + ((T - i) % B - b);
#pragma unroll
    for (int m = 8; m < 16; m++)
    {
      if (ABL == 3 || ABL == 1)
      {
        if (ABL == 1)
          v[m] = mir[(i == 0 ? 16 - m : 15 - m) * WG + tp];
      }
      else if (i == 0 && m == 8)
      {
        // Nyquist column: first column of the last strip
        const int off = RM ? r * rs.lp + rs.cpr : half_group_offset<LOGN, RG, FB>(y, N / 2 / FB);
        const int offc = RM ? off : half_group_offset<LOGN, RGC, FB>(y, N / 2 / FB);
        const size_t ns = RM ? (size_t)rs.nyq_src * rs.src_stride : 0;
        const float4* fab = RM ? reinterpret_cast<const float4*>(rs.ab + ns) + base : gab + base;
        const float4* fde = RM ? reinterpret_cast<const float4*>(rs.de + ns) + base : gde + base;
        const float2* fc = RM ? reinterpret_cast<const float2*>(rs.c + ns) + base : gc + base;
        const float kx = -(dim / 2.0f) * dk;
        float2 cc;
        if (BOTH && img == 1)
          cc = cnyq;
        else
          cc = ld2<LA>(fc, offc * 8);  // C
        if (BOTH && img == 0)
          cnyq = cc;
        if (img == 0)
        {
          const CPair p = raw_pair(ld4<LA>(fab, off * 16));  // (A, B)
          v[m] = CPair{f2v{(1.0f - kx) * p.re.x, -p.im.y - kx * cc.x},
                       f2v{(1.0f - kx) * p.im.x, p.re.y - kx * cc.y}};
        }
        else
        {
          const CPair q = raw_pair(ld4<LA>(fde, off * 16));  // (D, E): D = (re.x, im.x)
          const float kx2 = kx * kx;
          v[m] = CPair{f2v{-(q.im.x - kx2 * cc.y), -q.re.y + kx * q.im.x},
                       f2v{q.re.x - kx2 * cc.x, -q.im.y - kx * q.re.x}};
        }
      }
      else if constexpr (!XS)
        v[m] = mir[(i == 0 ? 16 - m : 15 - m) * WG + tp];
    }
    if constexpr (ABL != 3 && !XS)
      __syncthreads();  // the transform's first exchange reuses the LDS
    int i2 = opaque(i20), r2 = RPW == 1 ? 0 : opaque(r20);
    if constexpr (XS)
    {
      // x index n = n1 + 16 n2, output k = k2 + 1024 k1 (T = 1024): transposition T_in gives wave
      // n1 = w the inputs x(w + 16 n2) (own lanes at n, the -u lanes at N - n, thread 0's Nyquist
      // column at N/2); the wave's 1024-point sub-transform; times W_N^(n1 k2); transposition T_out
      // gives thread k2 = tid the 16 values Z_n1(k2); the 16-point DFT over n1 leaves
      // v[k1] = X(tid + T k1): the plain path's store layout. LDS slot of n: (n mod 16) RS + n / 16.
      constexpr int L2 = XsCfg<LOGN>::L2, RS = XsCfg<LOGN>::RS;
      const int w = tid >> 6, l = tid & 63;
      float2* xs = reinterpret_cast<float2*>(xch);
      auto pslot = [&](int n) { return (n & 15) * RS + (n >> 4); };
      __syncthreads();  // the previous image's T_out reads are done
#pragma unroll
      for (int h = 0; h < 2; h++)
      {
        if (h)
          __syncthreads();
#pragma unroll
        for (int m = 0; m < 8; m++)
        {
          xs[pslot(i + m * T)] = half_of(v[m], h);
          xs[pslot(m == 0 && i == 0 ? N / 2 : N - i - m * T)] = half_of(v[m + 8], h);
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < 16; m++)
          set_half(v[m], h, xs[w * RS + l + 64 * m]);
      }
      // region w is the wave's alone until T_out's first barrier: its exchanges need no barriers
      fft_run<L2, 0, true, true>(v, l, 0, l, 0, xs + w * RS, tw2);  // v[m] = Y_w(l + 64 m)
      const float2 base_w = twiddle<LOGN>(w * l, tw);
#pragma unroll
      for (int m = 0; m < 16; m++)
        v[m] = cmul(v[m], base_w);
      apply_stage_twiddles<LOGN>(v, 64 * w, tw);  // x W_N^(w (l + 64 m))
#pragma unroll
      for (int h = 0; h < 2; h++)
      {
        if (h)
          __syncthreads();
#pragma unroll
        for (int m = 0; m < 16; m++)
          xs[w * RS + l + 64 * m] = half_of(v[m], h);
        __syncthreads();
#pragma unroll
        for (int n1 = 0; n1 < 16; n1++)
          set_half(v[n1], h, xs[n1 * RS + tid]);
      }
      idft16(v);
      i2 = tid;
    }
    else if constexpr (ABL != 2)
      fft_run<LOGN, CI, true>(v, i, r, i2, r2, xch, tw);
    float4* dst = maps + ((size_t)cimg * (RM ? rows : N) + y0) * N;
    const int woff = ((r2 << LOGN) + i2) * 16;
#pragma unroll
    for (int m = 0; m < 16; m++)
      st4<SA>(dst + m * T, woff, from_pair(v[m]));
    if (img & 1)
    {
      // displacementMap (Dz, dDx/dx, dDz/dz, dDx/dz) = (re0, im0, re1, im1): Jacobian,
      // spectrum.compute:246-259
      const float lam = foam.displacement[c];
      float* jb = jac + ((size_t)c * (RM ? rows : N) + y0) * N;
      const int joff = ((r2 << LOGN) + i2) * 4;
#pragma unroll
      for (int m = 0; m < 16; m++)
        st1<SA>(jb + m * T, joff,
                (1.0f + lam * v[m].im.x) * (1.0f + lam * v[m].re.y) - lam * lam * v[m].im.y * v[m].im.y);
    }
    }
  }
}

}  // namespace oceanfft
