// device/k_fft.h — kernels of the standalone EncodeIFFT (src/FFTCalculator.cpp:73-114,
// resources/fft.compute:21-88) on caller-owned row-major RGBA32F images: the in-place row and column
// passes, the column-first strided pass of N = 4096, and the four-step column transform of N = 16384.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ocean_internal.h"
#include "device/fft.h"
#include "device/grid.h"
#include "device/memory.h"

namespace oceanfft
{

// ------------------------------------------------------------------------------------------------
// FFTCalculator::EncodeIFFT path on caller-owned row-major images: row pass then column pass,
// both in place (no work image).
// ------------------------------------------------------------------------------------------------
template <int LOGN>
struct RowCfg
{
  using S = FftShape<LOGN>;
  static constexpr int RPW = S::T >= 256 ? 1 : 256 / S::T;  // rows per workgroup iteration
  static constexpr int WG = S::T * RPW;
  static constexpr bool SPLIT = (S::N * 16 > 96 * 1024);   // float4 exchange would not fit
  static constexpr int LDS_BYTES = lds_row_slots<LOGN>(RPW) * (SPLIT ? 8 : 16);
  // waves per SIMD the LDS budget admits (>= 1): caps VGPRs so registers never limit residency
  static constexpr int WGS_PER_CU = (150 * 1024) / (LDS_BYTES + 2048) < 1 ? 1 : (150 * 1024) / (LDS_BYTES + 2048);
  static constexpr int MIN_WAVES_RAW = WGS_PER_CU * (WG / 64) / 4;
  static constexpr int MIN_WAVES = MIN_WAVES_RAW < 1 ? 1 : (MIN_WAVES_RAW > 8 ? 8 : MIN_WAVES_RAW);
};

// Row pass of a plain EncodeIFFT on packed images [n_images][N][N] float4, in place.
template <int LOGN>
__global__ __launch_bounds__(RowCfg<LOGN>::WG, RowCfg<LOGN>::MIN_WAVES) void k_rows_ifft(
    int rows, float4* __restrict__ images, const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  using R = RowCfg<LOGN>;
  constexpr int N = S::N, T = S::T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);

  const int rho0 = threadIdx.x / T, i0 = threadIdx.x % T;
  const int total = rows;  // rows of N packed texels, contiguous (n_images * N for whole images)
  for (int row0 = blockIdx.x * R::RPW; row0 < total; row0 += gridDim.x * R::RPW)
  {
    const int i = opaque(i0), rho = R::RPW == 1 ? 0 : opaque(rho0);
    // rows row0 .. row0+RPW-1 are contiguous: uniform base, lane offset (rho*N + i)*16; the
    // range limit zeroes/drops rows past the last image (ragged tail for small N)
    float4* lines = images + ((size_t)row0 << LOGN);
    const int lim = clamp_bytes((int64_t)(total - row0) * N * 16);
    const int voff = ((rho << LOGN) + i) * 16;
    CPair v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
      v[m] = to_pair(ld4(lines + ((m + 8) & 15) * T, voff, lim));  // fftShift on x folded into the load
    fft_run<LOGN, 0, R::SPLIT>(v, i, rho, xch, tw);
#pragma unroll
    for (int m = 0; m < 16; m++)
      st4(lines + m * T, voff, from_pair(v[m]), lim);
  }
}

// Column pass in place: strips of C texel columns, transformed along y.
// GROUP: consecutive strips on blocks b, b + 8, ... (one XCD, xcd_group_slot), so the partial lines
// of C-column pieces (C * 16 B) meet in one L2.
// CC: columns per strip (ColCfg's C by default: 16 at N <= 1024, one 1024-thread workgroup per strip).
// With few images a 1024^2 image has only 64 such strips for 256 CUs; launch_cols then takes CC = 4
// (256-thread workgroups, 256 strips per image), the same per-column arithmetic (round 6).
template <int LOGN, int GROUP = 2, int CC = ColCfg<LOGN>::C>
__global__ __launch_bounds__(FftShape<LOGN>::T * CC) void k_cols(int n_images, float4* __restrict__ images,
                                                                 const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  constexpr int T = S::T, C = CC, STRIPS = S::N / CC;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);

  const int c0 = threadIdx.x % C, i0 = threadIdx.x / C;
  const int total = n_images * STRIPS;
  for (int item = xcd_group_slot<GROUP>(blockIdx.x, gridDim.x); item < total; item += gridDim.x)
  {
    const int c = opaque(c0), i = opaque(i0);
    const int img = item / STRIPS, strip = item - img * STRIPS;
    const int x = strip * C + c;
    // image rows i + mm*T: uniform base per mm (SGPR), lane offset (i*N + x)*16 shared by all mm
    float4* ibase = images + ((size_t)img << (2 * LOGN));
    const int voff = ((i << LOGN) + x) * 16;
    CPair v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
    {
      // input q = i + m*T sits in row (q + N/2) mod N = i + ((m + 8) mod 16)*T: fftShift on y
      const int mm = (m + 8) & 15;
      v[m] = to_pair(ld4(ibase + ((size_t)(mm * T) << LOGN), voff));
    }
    fft_run<LOGN, C, true>(v, i, c, xch, tw);
#pragma unroll
    for (int m = 0; m < 16; m++)
      st4(ibase + ((size_t)(m * T) << LOGN), voff, from_pair(v[m]));
  }
}

// Standalone EncodeIFFT, column-first with a work image (src/FFTCalculator.cpp keeps a workImage
// too): pass A reads the caller's row-major image in strips of B columns (64-B pieces per row,
// the only strided access), iFFTs along y with the fftShift folded into the row index, and writes
// the blocked split-plane work image work[img][x/B][y][B] contiguously; pass B is k_rows_final on
// it (256-B runs in, row-major rows out, no Jacobian). Measured patterns (profiles/
// r01_colbench_patterns.log): strided read + contiguous write 3.4 TB/s, against 2.1-2.4 TB/s for
// the in-place column pass that reads and writes 64-B pieces.
// LA: default-policy loads. Each 128-B line is read half by this block and half by the block of
// the adjacent strip (same XCD, same time); streamed (nt) loads lost the line before the partner's
// read: 1.38 -> 1.12 ms per 8 images (tools/microbench/ifftbench; grouping 4 or 8 strips: no gain).
template <int LOGN, int LA = 0, int GROUP = 2>
__global__ __launch_bounds__(ColFirstCfg<LOGN>::WG1) void k_cols_to_blocks(int images, const float4* __restrict__ src_images,
                                                                          float4* __restrict__ work,
                                                                          const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  using K = ColFirstCfg<LOGN>;
  constexpr int N = S::N, T = S::T, B = K::B, SPW = K::SPW;
  static_assert(SPW == 1, "one strip per item");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);
  const int strips = N / B;
  const int total = images * strips;
  // adjacent strips (the two 64-B halves of each 128-B line) on blocks b, b+8: one XCD, one L2
  for (int item = xcd_group_slot<GROUP>(blockIdx.x, gridDim.x); item < total; item += gridDim.x)
  {
    const int tid = opaque((int)threadIdx.x);
    const int b = tid % B, i = (tid / B) % T;
    const int img = item / strips, xb = item - img * strips;
    // row y = i + mm*T of the input, column xb*B + b: uniform base per m, lane offset (i*N + b)*16
    const float4* src = src_images + ((size_t)img << (2 * LOGN)) + (size_t)xb * B;
    const int voff = ((i << LOGN) + b) * 16;
    CPair v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
      v[m] = to_pair(ld4<LA>(src + ((size_t)(((m + 8) & 15) * T) << LOGN), voff));  // fftShift on y
    fft_run<LOGN, K::C1, true>(v, i, b, xch, tw);
    float4* dst = work + ((size_t)img << (2 * LOGN)) + (size_t)xb * N * B;
    const int soff = (i * B + b) * 16;
#pragma unroll
    for (int m = 0; m < 16; m++)
      st4<kStream>(dst + m * T * B, soff, pair_raw(v[m]));
  }
}

// Standalone EncodeIFFT at N = R M, M = 4096 (R = 2: 8192, R = 4: 16384), column-first with a
// radix-R pre-stage, so that a column item is the 4096 pass's shape (a strip of B = 4 columns, 64-B
// pieces, 256 KiB of CPairs) instead of one or two whole columns (16/32-B pieces). With y index
// q = n + M j and k = R k' + r:
//   X[R k' + r] = sum_n W_M^(n k') [W_N^(n r) sum_j x[n + M j] W_R^(j r)],
// so item (strip, r) forms y_r[n] = W_N^(n r) sum_j x[n + M j] W_R^(j r) from R loads per point and
// runs the 4096-point transform, which leaves X[R k' + r] at k' = i + m T. The R items of a strip
// read the same lines and the two strips of a 128-B line share them: the 2R items run together on
// one XCD (xcd_group_slot), so HBM serves each line once and L2 the rest.
// WL (work layout): 0 = [img][strip][r][k'][B] split planes (each item writes one contiguous 256-KiB
// run; the row pass reads stored row r M + k' and writes image row R k' + r: k_rows_final PR); 1 =
// row-major [img][y][x] reference texels (64-B pieces of rows R k' + r; k_rows_ifft_out).
// The pre-stage sum in the wave-uniform r, branch-free (c = (-1)^r, w = i^r computed once per item):
// R = 2: x0 + c x1; R = 4: (x0 + c x2) + w (x1 + c x3) (inverse: W_4 = +i).
template <int R>
__device__ __forceinline__ CPair prestage_sum(const CPair* x, float c, float2 w)
{
  const f2v cc = {c, c};
  if constexpr (R == 2)
    return {x[0].re + cc * x[1].re, x[0].im + cc * x[1].im};
  else
  {
    static_assert(R == 4, "pre-stage radix 2 or 4");
    const CPair s02 = {x[0].re + cc * x[2].re, x[0].im + cc * x[2].im};
    const CPair t13 = {x[1].re + cc * x[3].re, x[1].im + cc * x[3].im};
    return s02 + cmul(t13, w);
  }
}

struct PreCfg
{
  static constexpr int LOGM = 12, M = 4096, T = 256, B = 4, WG = 1024;
  static constexpr int TWM = ((FftShape<LOGM>::TW_ENTRIES * 8 + 15) / 16) * 16;
  static constexpr int XCH = B * FftShape<LOGM>::PADDED * 8;
};

template <int LOGN, int LA = 0, int WL = 0, int LB = 2>
__global__ __launch_bounds__(PreCfg::WG) void k_cols_pre(int images, const float4* __restrict__ src_images,
                                                         float4* __restrict__ work, const float2* __restrict__ twn_glob,
                                                         const float2* __restrict__ twm_glob)
{
  using P = PreCfg;
  using SN = FftShape<LOGN>;
  constexpr int N = SN::N, M = P::M, R = N / M, T = P::T, B = P::B;
  static_assert(R == 2 || R == 4, "N = 8192 or 16384");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* twm = reinterpret_cast<float2*>(smem);
  float2* twn = reinterpret_cast<float2*>(smem + P::TWM);
  void* xch = smem + P::TWM + ((SN::TW_ENTRIES * 8 + 15) / 16) * 16;
  for (int e = threadIdx.x; e < SN::TW_ENTRIES; e += blockDim.x)
    twn[e] = twn_glob[e];
  load_twiddles<P::LOGM>(twm, twm_glob);
  const int strips = N / B;
  const int total = images * strips * R;
  // item = ((img strips/2 + strip pair) R + r) 2 + strip & 1: the 2R items sharing lines are consecutive
  for (int item = xcd_group_slot<2 * R>(blockIdx.x, gridDim.x); item < total; item += gridDim.x)
  {
    const int tid = opaque((int)threadIdx.x);
    const int b = tid & (B - 1), i = tid / B;
    const int it = __builtin_amdgcn_readfirstlane(item);  // keep the item math scalar (no waterfall loops)
    int t = it >> 1;
    const int r = t % R;
    t /= R;
    const int sp = t % (strips / 2), img = t / (strips / 2);
    const int xb = sp * 2 + (it & 1);
    const float c = (r & 1) ? -1.0f : 1.0f;
    const float2 w = make_float2((r & 1) ? 0.0f : c * (1.0f - (float)(r & 2)), (r & 1) ? 1.0f - (float)(r & 2) : 0.0f);
    const float4* src = src_images + ((size_t)img << (2 * LOGN)) + (size_t)xb * B;
    const int voff = ((i << LOGN) + b) * 16;
    CPair v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
    {
      CPair x[R];
#pragma unroll
      for (int j = 0; j < R; j++)  // q = i + m T + M j sits in row (q + N/2) mod N: fftShift on y
      {
        // one descriptor per image (64 per-piece descriptors spill SGPRs, then VGPRs): the row offset
        // joins the lane offset as an unsigned 32-bit byte offset (< 4 GiB = one 16384^2 image)
        const unsigned row = (unsigned)((m * T + j * M + N / 2) & (N - 1));
        x[j] = to_pair(ld4<LA>(src, (int)((unsigned)voff + (row << (LOGN + 4))), -1));
      }
      v[m] = cmul(prestage_sum<R>(x, c, w), twiddle<LOGN>((i + m * T) * r, twn));
      if (LB > 0 && (m & (LB - 1)) == LB - 1)
        asm volatile("" ::: "memory");  // LB points' loads in flight
    }
    fft_run<P::LOGM, B, true>(v, i, b, xch, twm);  // v[m] = X[R (i + m T) + r]
    if constexpr (WL == 0)
    {
      float4* dst = work + ((size_t)img << (2 * LOGN)) + (size_t)(xb * R + r) * M * B;
      const int soff = (i * B + b) * 16;
#pragma unroll
      for (int m = 0; m < 16; m++)
        st4<kStream>(dst + m * T * B, soff, pair_raw(v[m]));
    }
    else
    {
      float4* dst = work + ((size_t)img << (2 * LOGN)) + (size_t)xb * B;
      const int soff = (((R * i) << LOGN) + b) * 16;
#pragma unroll
      for (int m = 0; m < 16; m++)
        st4<kStream>(dst + ((size_t)(R * m * T + r) << LOGN), soff, from_pair(v[m]));
    }
  }
}

// Row pass from a row-major work image to the caller's image (WL = 1 above): k_rows_ifft with
// separate source and destination.
template <int LOGN>
__global__ __launch_bounds__(RowCfg<LOGN>::WG, RowCfg<LOGN>::MIN_WAVES) void k_rows_ifft_out(
    int rows, const float4* __restrict__ src, float4* __restrict__ dst, const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  using R = RowCfg<LOGN>;
  constexpr int T = S::T;
  static_assert(R::RPW == 1, "one row per item");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);
  for (int row = blockIdx.x; row < rows; row += gridDim.x)
  {
    const int i = opaque((int)threadIdx.x % T);
    const float4* in = src + ((size_t)row << LOGN);
    float4* out = dst + ((size_t)row << LOGN);
    CPair v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
      v[m] = to_pair(ld4<kStream>(in + ((m + 8) & 15) * T, i * 16));  // fftShift on x
    fft_run<LOGN, 0, R::SPLIT>(v, i, 0, xch, tw);
#pragma unroll
    for (int m = 0; m < 16; m++)
      st4<kStream>(out + m * T, i * 16, from_pair(v[m]));
  }
}

// Standalone EncodeIFFT at N >= 8192: the column transform in four steps (N = 16 N2), so that no
// access is a 16- or 32-byte column piece (one 16384-row column is 256 KiB: an in-place column
// item holds one or two columns and reads 16-32-B pieces, 1.3-2.8 TB/s). For y index n = N2 n1 + n2
// and k = k1 + 16 k2:  X[k1 + 16 k2] = sum_n2 W_N2^(n2 k2) [W_N^(n2 k1) sum_n1 x[N2 n1 + n2] W_16^(n1 k1)].
// Step 1 (this kernel), per (column x, n2): the 16-point inverse DFT over rows N2 n1 + n2 (fftShift
// on y folded into n1: row (n + N/2) mod N = N2 ((n1 + 8) mod 16) + n2), times W_N^(n2 k1), into the
// work slab at row N2 k1 + n2, split planes. Lanes run along x: every load and store of a wave is one
// 1-KiB row piece, and there is no LDS exchange. The work slab holds columns [x0, x0 + wc).
// WNT: the work slab's stores (here) and loads (step 2) non-temporal (production). false: default
// policy, so that a slab of <= 128 MiB could stay in the Infinity Cache between the two steps: measured
// and not kept (2 x 16384^2: 10.02 ms at best, slab 1024 columns, against 10.00 for 2048 nt;
// profiles/r04_ifft4bench_mall.log).
// MINW: the launch bound's minimum waves per SIMD; 4 keeps the kernel at <= 128 VGPRs, so four of its
// one-wave-per-SIMD workgroups share a CU (without it: 138 VGPRs, three).
template <int LOGN, bool WNT = true, int MINW = 4>
__global__ __launch_bounds__(256, MINW) void k_cols4_step1(int images, int x0, int wc, const float4* __restrict__ img,
                                                     float4* __restrict__ work, const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  constexpr int N = S::N, N2 = N / 16;
  __shared__ float2 tw[S::TW_ENTRIES];
  load_twiddles<LOGN>(tw, tw_glob);
  const int xblocks = wc / 64;
  const int total = images * xblocks * (N2 / 4);
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int t = item;
    const int xbk = t % xblocks;
    t /= xblocks;
    const int n2 = (t % (N2 / 4)) * 4 + wv, im = t / (N2 / 4);
    const int xl = xbk * 64 + lane;  // column within the slab
    const float4* src = img + ((size_t)im << (2 * LOGN)) + x0 + xl;
    CPair v[16];
#pragma unroll
    for (int n1 = 0; n1 < 16; n1++)
    {
      const f4v r = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(src + (size_t)(N2 * ((n1 + 8) & 15) + n2) * N));
      v[n1] = to_pair(make_float4(r.x, r.y, r.z, r.w));
    }
    idft16(v);
    apply_stage_twiddles<LOGN>(v, n2, tw);  // v[k1] *= W_N^(n2 k1)
    float4* dst = work + (size_t)im * N * wc + xl;
#pragma unroll
    for (int k1 = 0; k1 < 16; k1++)
    {
      const float4 o = pair_raw(v[k1]);
      if constexpr (WNT)
        __builtin_nontemporal_store(f4v{o.x, o.y, o.z, o.w}, reinterpret_cast<f4v*>(dst + (size_t)(N2 * k1 + n2) * wc));
      else
        dst[(size_t)(N2 * k1 + n2) * wc] = o;
    }
  }
}

// Step 2, per (image, k1, strip of C slab columns): the N2-point inverse FFT along the work slab's
// contiguous rows N2 k1 + n2 (n2 = i + m T), output X[k1 + 16 k2] to image row k1 + 16 k2 in the
// reference layout. Loads and stores are C * 16 = 256-byte row pieces. tw_glob: the N2-point table.
// CI: columns per workgroup (ColCfg's 16 = 1024 threads at N2 = 1024, production; 8 = 512 threads, two
// per CU, as k_gen4_step2: 10.62 against 10.00 ms for 2 x 16384^2, tools/microbench/ifft4bench ci).
// Round 6: the item's source address and the lane offsets are formed per load from opaque() values
// (src_of / ld), which keeps the kernel at 112 VGPRs; the earlier form spilled 8 VGPRs (36 B) at the
// 128 of a 1024-thread workgroup. 2 x 16384^2: 10.009 -> 9.753 ms on one box (ifft4bench early,
// profiles/r06_ifft4bench_early2.log), bit-identical.
// MINW (round 6): the launch bound's minimum waves per SIMD. CI 8 needs 4 for two 512-thread workgroups
// per CU: without it the kernel compiles to 134 VGPRs and only one fits (round 5's CI 8 measurement).
template <int LOGN2, bool WNT = true, int CI = ColCfg<LOGN2>::C, int MINW = (CI < ColCfg<LOGN2>::C ? 4 : 1)>
__global__ __launch_bounds__(FftShape<LOGN2>::T * CI, MINW) void k_cols4_step2(int images, int x0, int wc,
                                                                        const float4* __restrict__ work,
                                                                        float4* __restrict__ img,
                                                                        const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN2>;
  constexpr int N2 = S::N, T = S::T, C = CI, LOGN = LOGN2 + 4, N = N2 * 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN2>(tw, tw_glob);
  const int c0 = threadIdx.x % C, i0 = threadIdx.x / C;
  const int strips = wc / C;
  const int total = images * 16 * strips;
  auto src_of = [&](int item) __attribute__((always_inline)) {
    const int strip = item % strips, rest = item / strips, k1 = rest & 15, im = rest >> 4;
    return work + (size_t)im * N * wc + (size_t)N2 * k1 * wc + strip * C + opaque(c0);
  };
  auto ld = [&](const float4* src, int m) __attribute__((always_inline)) {
    const float4* p = src + (size_t)(opaque(i0) + m * T) * wc;
    if constexpr (WNT)
    {
      const f4v r = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
      return raw_pair(make_float4(r.x, r.y, r.z, r.w));
    }
    else
      return raw_pair(*p);
  };
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    const int c = opaque(c0), i = opaque(i0);
    const int strip = item % strips, rest = item / strips, k1 = rest & 15, im = rest >> 4;
    const int xl = strip * C + c;
    const float4* src = src_of(item);
    CPair v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
      v[m] = ld(src, m);
    fft_run<LOGN2, C, true>(v, i, c, xch, tw);
    float4* dst = img + ((size_t)im << (2 * LOGN)) + (size_t)k1 * N + x0 + xl;
#pragma unroll
    for (int m = 0; m < 16; m++)
    {
      const float4 o = from_pair(v[m]);
      __builtin_nontemporal_store(f4v{o.x, o.y, o.z, o.w},
                                  reinterpret_cast<f4v*>(dst + (size_t)16 * (i + m * T) * N));
    }
  }
}

}  // namespace oceanfft
