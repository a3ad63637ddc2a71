// device/k_rows_hp.h — the half-spectrum row pass of whole 4096^2 grids (blocked field layout) with
// the x transform split 16 x 256: one LDS transposition T_in that also does the mirror exchange, the
// 256-point sub-transforms inside the wave (lane_xchg.h: v_permlane16/32_swap + DPP), a second
// transposition T_out, a 16-point DFT in registers. Production k_rows_half moves the -u lanes through
// the LDS, then runs fft_run<12> with two split exchanges: 2.5 LDS round trips and 10 barriers per
// image against 2 and 7 here.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ocean_internal.h"
#include "device/fft.h"
#include "device/grid.h"
#include "device/k_half_cols.h"
#include "device/lane_xchg.h"
#include "device/memory.h"

namespace oceanfft
{

// x index n = n1 + 16 n2 (n1 < 16, n2 < 256), output k = k2 + 256 k1:
//   X(k2 + 256 k1) = sum_n1 W_16^(n1 k1) [W_N^(n1 k2) Y_n1(k2)],  Y_n1(k2) = sum_n2 x(n1 + 16 n2) W_256^(n2 k2).
// LDS slot of (n1, j), 8-B halves: n1 RS + (j ^ g(n1)), RS = 8 (mod 32), g(n1) = ((n1 >> 1) & 7) ^
// (((n1 >> 1) & 1) << 2). MI355X_MICROARCH.md §LDS banks ds_write_b64 in 16-lane groups (8-B slot mod 16)
// and ds_read_b64 in 32-lane groups (slot mod 32); with this layout all four access shapes are
// conflict-free: T_in's writes (16 consecutive n1 at one j), T_in's reads and T_out's writes (4 n1 of
// one wave x 8 or 4 consecutive j), T_out's reads (32 consecutive j at one n1). (RS = 260 with the XOR
// of (n1 >> 2) & 3 left T_in's reads 2-way; tools/xp_model.py checks the bank multiplicities.)
struct HpCfg
{
  static constexpr int LOGN = 12, RS = 264;
  static constexpr int TW = ((FftShape<LOGN>::TW_ENTRIES * 8 + 15) / 16) * 16;
  static constexpr int LDS = TW + 16 * RS * 8;
};

__device__ __forceinline__ int hp_swz(int n1) { return ((n1 >> 1) & 7) ^ (((n1 >> 1) & 1) << 2); }
__device__ __forceinline__ int hp_slot(int n1, int j) { return n1 * HpCfg::RS + (j ^ hp_swz(n1)); }

// One row (both images; C loaded once, kept for image 1) per 256-thread workgroup, four per CU, the
// 4 rows of a gc line on one XCD; default-policy loads, streamed stores (production k_rows_half's
// item shape at 4096). RM: the fields are row-major behind a RowSrc (the strip-dealt slabs' row pass,
// rows = the rank's rows; streamed loads, C loaded per image, one row per workgroup in order), so slab
// frames stay bit-identical to whole grids.
//   T_in: thread (w, s, p) = (tid >> 6, tid & 3, (tid >> 2) & 15) receives x(n1 + 16 (p + 16 m)),
//         n1 = 4 w + s (four 256-point sub-transforms per wave).
//   sub-transform as k_rows_xp: v[b] = Y_n1(p + 16 b), then x W_N^(n1 (p + 16 b)).
//   T_out: thread k2 = tid receives Z_n1(k2), n1 < 16; DFT-16: v[k1] = X(tid + 256 k1).
// YP: the fields hold row y at storage row hx_store_row(y) (k_cols_half HX 2); items run over storage
// rows, so the 4 rows of a gc line stay on one XCD. FB: field strips of FB columns (k_cols_half FB);
// GRP: consecutive rows per XCD group (the rows of a gc line).
// EARLY (round 5, as k_rows_xs EARLY): a wave retires its memory instructions in issue order, so loads
// issued after an image's 16 map stores wait for those stores. 1: image 1's (D, E) loads are issued
// before image 0's stores (32 VGPRs from the end of image 0's transform to image 1's T_in); 2: and
// the next row's (A, B) and C before image 1's stores (the first row's in a prologue; persistent
// grids); whole grids only.
// MINB: the workgroups per CU the launch bounds ask for (4: 128 VGPRs; 3: 168, room for EARLY 2's
// prefetch without spills).
template <int RG, int RGC, bool RM = false, bool YP = false, int FB = 4, int GRP = 4, int EARLY = 0, int MINB = 4>
__global__ __launch_bounds__(256, MINB) void k_rows_hp(FrameParams fp, const float4* __restrict__ gab,
                                                 const float4* __restrict__ gde, const float2* __restrict__ gc,
                                                 const float4* __restrict__ spec, float4* __restrict__ maps,
                                                 float* __restrict__ jac, FoamParams foam,
                                                 const float2* __restrict__ tw_glob, int rows, RowSrc rs)
{
  constexpr int LOGN = HpCfg::LOGN, RS = HpCfg::RS;
  using S = FftShape<LOGN>;
  using HC = HalfCfg<LOGN>;
  constexpr int N = S::N, T = S::T, B = 4, STRIPS = HC::STRIPS;
  static_assert(T == 256, "one 4-wave row per workgroup");
  static_assert(!(RM && YP), "storage-row order is a whole-grid layout");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  float2* xs = reinterpret_cast<float2*>(smem + HpCfg::TW);
  load_twiddles<LOGN>(tw, tw_glob);

  const int nrows = RM ? rows : N;
  const int total = fp.cascades * nrows;
  const float dim = (float)N;
  constexpr int LA = RM ? kStream : 0;
  const int lcpr = RM ? 31 - __builtin_clz(rs.cpr) : 0, cmask = RM ? rs.cpr - 1 : 0;
  const int wave0 = __builtin_amdgcn_readfirstlane((int)threadIdx.x & ~63);
  static_assert(!EARLY || !RM, "EARLY: whole-grid layouts");
  float4 fpre[EARLY > 0 ? 8 : 1];  // EARLY: the next image's field texels, issued before the stores
  float2 cpre[EARLY >= 2 ? 8 : 1];  // EARLY 2: the next row's C
  // the field texels of image img of row item (whole grids), into f (and C into cdst)
  auto issue = [&](int item, int img, float4* f, float2* cdst) __attribute__((always_inline)) {
    const int c = item / nrows, yf = item - c * nrows;
    const size_t base = (size_t)c * STRIPS * N * B;
    const int i = opaque((int)threadIdx.x);
#pragma unroll
    for (int m = 0; m < 8; m++)
    {
      const int u = m * T + i;
      f[m] = ld4<LA>((img == 0 ? gab : gde) + base, half_group_offset<LOGN, RG, FB>(yf, u / FB, u % FB) * 16);
      if (cdst)
        cdst[m] = ld2<0>(gc + base, half_group_offset<LOGN, RGC, FB>(yf, u / FB, u % FB) * 8);
    }
  };
  const int item0 = RM ? (int)blockIdx.x : xcd_group_slot<GRP>(blockIdx.x, gridDim.x);
  if (EARLY >= 2 && item0 < total)
    issue(item0, 0, fpre, cpre);
  for (int item = item0; item < total; item += gridDim.x)
  {
    const int c = item / nrows, yf = item - c * nrows;  // RM: yf is the local row (slabs start at an even row)
    const int y = YP ? hx_row_of_store(yf) : yf;       // the output row; yf addresses the fields
    const float dk = fp.c[c].dk;
    const size_t base = RM ? ((size_t)c * rows + y) * rs.lp : (size_t)c * STRIPS * N * B;
    const float sgy = (y & 1) ? -1.0f : 1.0f;
    float2 ckeep[8], cnyq;
#pragma unroll
    for (int img = 0; img < 2; img++)
    {
      const int cimg = c * 2 + img;
      const float4* sp = spec + (size_t)cimg * N;
      const int tid = opaque((int)threadIdx.x), i = tid;
      CPair v[16];  // own lanes in v[m], the -u lanes in v[m + 8] until T_in
#pragma unroll
      for (int m = 0; m < 8; m++)
      {
        const int u = m * T + i;
        // RM: source block of column u (wave-uniform, a scalar shift) and the element in its row
        const int src = RM ? (m * T + sopaque(wave0)) >> lcpr : 0;
        const int off = RM ? (u & cmask) : half_group_offset<LOGN, RG, FB>(yf, u / FB, u % FB);
        const int offc = RM ? off : half_group_offset<LOGN, RGC, FB>(yf, u / FB, u % FB);
        const float4* fab = RM ? reinterpret_cast<const float4*>(rs.ab + (size_t)src * rs.src_stride) : gab;
        const float4* fde = RM ? reinterpret_cast<const float4*>(rs.de + (size_t)src * rs.src_stride) : gde;
        const float2* fc = RM ? reinterpret_cast<const float2*>(rs.c + (size_t)src * rs.src_stride) : gc;
        const float kx = (float)u * dk;
        const float4 s4 = ld4<0>(sp, (N / 2 - u) * 16);
        if (img == 0)
        {
          const CPair p = raw_pair(EARLY >= 2 ? fpre[m] : ld4<LA>(fab + base, off * 16));
          const float2 cc = EARLY >= 2 ? cpre[m] : ld2<0>(fc + base, offc * 8);
          if constexpr (!RM)
            ckeep[m] = cc;
          const float Ar = p.re.x, Ai = p.im.x, Br = p.re.y, Bi = p.im.y, Cr = cc.x, Ci = cc.y;
          v[m] = CPair{f2v{(1.0f - kx) * Ar, -Bi - kx * Cr}, f2v{(1.0f - kx) * Ai, Br - kx * Ci}};
          v[m + 8] = CPair{f2v{(1.0f + kx) * Ar + sgy * s4.x, -Bi + kx * Cr + sgy * s4.z},
                           f2v{-(1.0f + kx) * Ai + sgy * s4.y, -Br - kx * Ci + sgy * s4.w}};
        }
        else
        {
          const CPair q = raw_pair(EARLY > 0 ? fpre[m] : ld4<LA>(fde + base, off * 16));
          // RM: C again (its second read, a few microseconds after the first, comes from L2): keeping
          // it beside the source-block addressing spills
          float2 cc;
          if constexpr (RM)
            cc = ld2<0>(fc + base, offc * 8);
          else
            cc = ckeep[m];
          const float Cr = cc.x, Ci = cc.y, Dr = q.re.x, Di = q.im.x, Er = q.re.y, Ei = q.im.y;
          const float kx2 = kx * kx;
          v[m] = CPair{f2v{-(Di - kx2 * Ci), -Er + kx * Di}, f2v{Dr - kx2 * Cr, -Ei - kx * Dr}};
          v[m + 8] = CPair{f2v{-(Di + kx2 * Ci) + sgy * s4.x, -Er - kx * Di + sgy * s4.z},
                           f2v{-Dr - kx2 * Cr + sgy * s4.y, Ei - kx * Dr + sgy * s4.w}};
        }
      }
      if (i == 0)
      {
        // the Nyquist column u = -N/2 (first column of the last strip; RM: block nyq_src, column cpr)
        // replaces the unused -u lane of u = 0
        const int off = RM ? rs.cpr : half_group_offset<LOGN, RG, FB>(yf, N / 2 / FB);
        const int offc = RM ? off : half_group_offset<LOGN, RGC, FB>(yf, N / 2 / FB);
        const size_t ns = RM ? (size_t)rs.nyq_src * rs.src_stride : 0;
        const float4* fab = RM ? reinterpret_cast<const float4*>(rs.ab + ns) : gab;
        const float4* fde = RM ? reinterpret_cast<const float4*>(rs.de + ns) : gde;
        const float2* fc = RM ? reinterpret_cast<const float2*>(rs.c + ns) : gc;
        const float kx = -(dim / 2.0f) * dk;
        if (RM || img == 0)
          cnyq = ld2<0>(fc + base, offc * 8);
        const float2 cc = cnyq;
        if (img == 0)
        {
          const CPair p = raw_pair(ld4<LA>(fab + base, off * 16));
          v[8] = CPair{f2v{(1.0f - kx) * p.re.x, -p.im.y - kx * cc.x}, f2v{(1.0f - kx) * p.im.x, p.re.y - kx * cc.y}};
        }
        else
        {
          const CPair q = raw_pair(ld4<LA>(fde + base, off * 16));
          const float kx2 = kx * kx;
          v[8] = CPair{f2v{-(q.im.x - kx2 * cc.y), -q.re.y + kx * q.im.x}, f2v{q.re.x - kx2 * cc.x, -q.im.y - kx * q.re.x}};
        }
      }
      // ---- T_in (own lanes at n = i + m T, the -u lanes at N - n, thread 0's v[8] at N/2)
      const int w = tid >> 6, l = tid & 63, s = l & 3, p = l >> 2;
      const int n1r = 4 * w + s;
      const int rd = n1r * RS + (p ^ hp_swz(n1r));  // + 16 m: x(n1r + 16 (p + 16 m))
      const int wo = hp_slot(i & 15, i >> 4);   // + 16 m
      const int nm = N - i;
      const int wm = hp_slot(nm & 15, nm >> 4);  // - 16 m
      const int wm0 = i == 0 ? hp_slot(0, (N / 2) >> 4) : wm;
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
      // ---- the 256-point sub-transform of n1r in the wave's registers
      idft16(v);
      apply_stage_twiddles<LOGN>(v, 16 * p, tw);  // x W_256^(p a) = W_N^(16 p a)
      transpose_reg_lanes_2_5(v);
      idft16(v);                                  // v[b] = Y_n1r(p + 16 b)
      const float2 base_w = twiddle<LOGN>(n1r * p, tw);
#pragma unroll
      for (int m = 0; m < 16; m++)
        v[m] = cmul(v[m], base_w);
      apply_stage_twiddles<LOGN>(v, 16 * n1r, tw);  // x W_N^(n1r (p + 16 b))
      // ---- T_out: thread k2 = tid gathers Z_n1(k2)
#pragma unroll
      for (int h = 0; h < 2; h++)
      {
        if (h)
          __syncthreads();
#pragma unroll
        for (int m = 0; m < 16; m++)
          xs[rd + 16 * m] = half_of(v[m], h);
        __syncthreads();
#pragma unroll
        for (int n1 = 0; n1 < 16; n1++)
          set_half(v[n1], h, xs[n1 * RS + (tid ^ hp_swz(n1))]);
      }
      idft16(v);  // v[k1] = X(tid + T k1)
      if constexpr (EARLY > 0)
      {
        if (img == 0)
          issue(item, 1, fpre, nullptr);
        else if constexpr (EARLY >= 2)
        {
          // unconditional (the last row re-reads its own image 0) so that the consumed registers are
          // not kept as the loop's other incoming value
          const int nx = item + (int)gridDim.x < total ? item + (int)gridDim.x : item;
          issue(nx, 0, fpre, cpre);
        }
      }
      float4* dst = maps + ((size_t)cimg * nrows + y) * N;
#pragma unroll
      for (int m = 0; m < 16; m++)
        st4<kStream>(dst + m * T, tid * 16, from_pair(v[m]));
      if (img == 1)
      {
        const float lam = foam.displacement[c];
        float* jb = jac + ((size_t)c * nrows + y) * N;
#pragma unroll
        for (int m = 0; m < 16; m++)
          st1<kStream>(jb + m * T, tid * 4,
                       (1.0f + lam * v[m].im.x) * (1.0f + lam * v[m].re.y) - lam * lam * v[m].im.y * v[m].im.y);
      }
    }
  }
}

}  // namespace oceanfft
