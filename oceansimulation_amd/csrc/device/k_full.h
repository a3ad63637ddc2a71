// device/k_full.h — the full-spectrum generator frame (116 B per point): k_cols_evolve (evolve
// + pack + y iFFT of both packed images) and k_rows_final (x iFFT + maps + Jacobian), the latter also
// the row pass of the column-first EncodeIFFT at N = 4096.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ocean_internal.h"
#include "device/evolve.h"
#include "device/fft.h"
#include "device/grid.h"
#include "device/memory.h"

namespace oceanfft
{

// KEEP: how many of the thread's 16 evolved amplitudes H (2 VGPRs each) stay live from the first
// packed image to the second; the rest are re-read from h0 (bytes this workgroup read ~20 us
// earlier) and evolved again. KEEP = 16 does not fit the 128 VGPRs of a 1024-thread workgroup at
// N = 4096 (spills, which cost HBM traffic); KEEP = 4 does (default_keep).
template <int LOGN, int KEEP, int LA = kStream, int SA = kStream, bool NOMEM = false, int LR = 0, bool NOCOMP = false>
__global__ __launch_bounds__(ColFirstCfg<LOGN>::WG1) void k_cols_evolve(
    FrameParams fp, SlabGeom g, const float4* __restrict__ h0, float4* __restrict__ inter,
    const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  using K = ColFirstCfg<LOGN>;
  constexpr int N = S::N, T = S::T, B = K::B, SPW = K::SPW;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);

  const int w = g.w, wb = g.w / B;  // slab columns (= rows per destination block), strips in slab
  const int groups = wb / SPW;      // pass-1 items per cascade
  const int total = fp.cascades * groups;
  const float dim = (float)N;
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    // thread coordinates re-derived from one opaque copy of threadIdx.x (fewer live VGPRs)
    const int tid = opaque((int)threadIdx.x);
    const int b = tid % B, sl = SPW == 1 ? 0 : tid / (B * T);
    const int c = item / groups, xb0 = (item - c * groups) * SPW;
    const CascadeFrame f = fp.c[c];
    // this item's SPW strips of the slab's h0 are one contiguous run of SPW*N*B texels
    const float4* src = h0 + ((size_t)c * wb + xb0) * N * B;
    const int x = g.x0 + (xb0 + sl) * B + b;  // global column (k index)
    float2 H[KEEP > 0 ? KEEP : 1];
#pragma unroll 1
    for (int img = 0; img < 2; img++)
    {
      // keep the k-vector math inside this iteration (see opaque())
      const int i = (opaque((int)threadIdx.x) / B) % T;
      const int voff = ((sl * N + i) * B + b) * 16;
      float4 a[16];
#pragma unroll
      for (int m = 0; m < 16; m++)
        if (img == 0 || m >= KEEP)
        {
          if constexpr (NOMEM)  // compute-only timing variant (microbench): no HBM reads
            a[m] = make_float4(1e-3f * m, 2e-3f * (float)i, 1e-3f * (float)b, 1e-4f * (float)item);
          else if (m < KEEP)  // read once per frame
            a[m] = ld4s<LA>(src, voff, ((m + 8) & 15) * T * B * 16);  // fftShift on y folded into the load
          else  // read twice (re-evolved for the second image): policy LR
            a[m] = ld4<LR>(src + ((m + 8) & 15) * T * B, voff);
        }
      CPair v[16];
#pragma unroll
      for (int m = 0; m < 16; m++)
      {
        const int y = i + ((m + 8) & 15) * T;
        KVec q = make_kvec(x, y, dim, f.dk);
        float2 Hm;
        if constexpr (NOCOMP)  // memory-only timing ablation (microbench): no evolution, no FFT
        {
          v[m] = CPair{f2v{a[m].x, a[m].y}, f2v{a[m].z, a[m].w}};
          continue;
        }
        if (img == 1 && m < KEEP)
          Hm = H[m];
        else
          Hm = evolve(a[m], q.k, f);
        if (img == 0 && m < KEEP)
          H[m] = Hm;
        v[m] = img == 0 ? pack_height(Hm, q) : pack_displacement(Hm, q);
      }
      if constexpr (!NOCOMP)
        fft_run<LOGN, K::C1, true>(v, i, sl * B + b, xch, tw);
      // Output rows y = i + m*T go to destination block q = y / w (uniform per m since T | w),
      // laid out inter[c][q][img][xb_local][y - q*w][B]: each destination's block is one
      // contiguous range (what the all-to-all sends; for ranks == 1 it is [c][img][xb][y][B]).
      float4* dst = inter + (size_t)c * 2 * N * w;
      const int soff = ((sl * w + i) * B + b) * 16;
#pragma unroll
      for (int m = 0; m < 16; m++)
      {
        const int q = (m * T) / w, yl = (m * T) % w;
        if constexpr (NOMEM)
          asm volatile("" ::"v"(v[m].re), "v"(v[m].im));
        else  // intermediate texels stay in split form (pair_raw): pass 2 reads them as such
          st4<SA>(dst + (((size_t)(q * 2 + img) * wb + xb0) * w + yl) * B, soff, pair_raw(v[m]));
      }
    }
  }
}

// BLOCKED: input is pass 1's output after the exchange, inter[c][src][img][xb_local][y][B] for this
// rank's w rows (xb = src * (w/B) + xb_local); otherwise row-major [c][img][y][x] (after
// k_blocks_to_rows, used when B == 1).
// ABL: timing ablations for tools/microbench (results wrong by construction): 1 = no HBM traffic,
// 2 = no FFT (memory traffic and stores only).
// GRPR (blocked input): consecutive items run on one XCD in groups of GRPR (xcd_group_slot), for a
// block width whose 128-B lines span more rows than one item reads (B = 2, RPW = 2: a line is 4 rows).
// BO: block width override (0: ColFirstCfg's B). PR > 1 (EncodeIFFT with k_cols_pre, WL = 0): stored
// row y' = r M + k' (M = N / PR) is image row PR k' + r.
template <int LOGN, bool BLOCKED, int LA = kStream, int SA = kStream, int RPW_ = ColFirstCfg<LOGN>::RPW2, int ABL = 0,
          int GRPR = 1, int BO = 0, int PR = 1>
__global__ __launch_bounds__(FftShape<LOGN>::T * RPW_) void k_rows_final(
    int images, SlabGeom g, const float4* __restrict__ inter, float4* __restrict__ maps, float* __restrict__ jac,
    FoamParams foam, const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  using K = ColFirstCfg<LOGN>;
  constexpr int N = S::N, T = S::T, B = BLOCKED ? (BO ? BO : K::B) : 1, RPW = RPW_;
  static_assert(PR == 1 || (BLOCKED && (N / PR) % RPW == 0), "PR: blocked input, items inside one r block");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);

  const int w = g.w, wb = g.w / B;
  const int blocks = w / RPW;  // pass-2 items per image
  // Loads (blocked input): lanes b fastest, then row r, then ihi, so 16 consecutive lanes read one
  // B*RPW*16-byte run [xb][y0..y0+RPW-1][0..B-1]. After the first exchange the thread becomes
  // position i2 of row r2 with i2 fastest, so each wave stores 64 consecutive texels of one row.
  // Row-major input: i fastest for both.
  const int b0 = threadIdx.x % B, r0 = (threadIdx.x / B) % RPW, ihi0 = threadIdx.x / (B * RPW);
  const int i20 = threadIdx.x % T, r20 = threadIdx.x / T;
  constexpr bool REMAP = BLOCKED && S::NSTAGE > 1;
  const int total = images * blocks;  // images = 2 per cascade (height, displacement)
  for (int item = GRPR > 1 ? xcd_group_slot<GRPR>(blockIdx.x, gridDim.x) : blockIdx.x; item < total;
       item += gridDim.x)
  {
    int i, r;
    if constexpr (BLOCKED)
    {
      const int b = opaque(b0), ihi = opaque(ihi0);
      r = RPW == 1 ? 0 : opaque(r0);
      i = ihi * B + b;
    }
    else
    {
      i = opaque(i20);
      r = RPW == 1 ? 0 : opaque(r20);
    }
    const int i2 = REMAP ? opaque(i20) : i, r2 = REMAP ? (RPW == 1 ? 0 : opaque(r20)) : r;
    const int cimg = item / blocks, y0 = (item - cimg * blocks) * RPW;
    const int c = cimg >> 1, img = cimg & 1;
    CPair v[16];
    if constexpr (BLOCKED)
    {
      const float4* src = inter + (size_t)c * 2 * N * w + (size_t)y0 * B;
      const int ihi = i / B, b = i % B;
      const int voff = ((ihi * w + r) * B + b) * 16;
#pragma unroll
      for (int m = 0; m < 16; m++)
      {
        // column block xb = ihi + mm*T/B: source rank and local block are uniform per m
        const int xbm = ((m + 8) & 15) * (T / B);  // fftShift on x
        const int srcr = xbm / wb, xbl = xbm % wb;
        if constexpr (ABL == 1)
          v[m] = CPair{f2v{1e-3f * m, (float)i}, f2v{(float)r, 1e-4f * (float)item}};
        else
          v[m] = raw_pair(ld4<LA>(src + ((size_t)(srcr * 2 + img) * wb + xbl) * w * B, voff));
      }
    }
    else
    {
      const float4* src = inter + ((size_t)cimg * w + y0) * N;
      const int voff = ((r << LOGN) + i) * 16;
#pragma unroll
      for (int m = 0; m < 16; m++)
        v[m] = raw_pair(ld4<LA>(src + ((m + 8) & 15) * T, voff));  // fftShift on x
    }
    if constexpr (ABL != 2)
      fft_run<LOGN, 0, true>(v, i, r, i2, r2, xch, tw);
    // PR: rows y0 + r2 of one r block are image rows PR (y0 mod M + r2) + y0 / M
    float4* dst = maps + ((size_t)cimg * w + (PR > 1 ? (y0 % (N / PR)) * PR + y0 / (N / PR) : y0)) * N;
    const int woff = (((r2 * PR) << LOGN) + i2) * 16;
#pragma unroll
    for (int m = 0; m < 16; m++)
      if constexpr (ABL == 1)
        asm volatile("" ::"v"(v[m].re), "v"(v[m].im));
      else
        st4<SA>(dst + m * T, woff, from_pair(v[m]));
    if (jac != nullptr && (img & 1))  // jac == nullptr: plain EncodeIFFT (launch_ifft_colfirst)
    {
      // displacementMap (Dz, dDx/dx, dDz/dz, dDx/dz) = (re0, im0, re1, im1): Jacobian,
      // spectrum.compute:246-259
      const float lam = foam.displacement[c];
      float* jb = jac + ((size_t)c * w + y0) * N;
      const int joff = ((r2 << LOGN) + i2) * 4;
#pragma unroll
      for (int m = 0; m < 16; m++)
      {
        const float jv = (1.0f + lam * v[m].im.x) * (1.0f + lam * v[m].re.y) - lam * lam * v[m].im.y * v[m].im.y;
        if constexpr (ABL == 1)
          asm volatile("" ::"v"(jv));
        else
          st1<SA>(jb + m * T, joff, jv);
      }
    }
  }
}

}  // namespace oceanfft
