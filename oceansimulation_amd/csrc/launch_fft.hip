// launch_fft.hip — the standalone EncodeIFFT (src/FFTCalculator.cpp:73-114) on caller-owned
// row-major images, and the full-spectrum generator frame (116 B per point). Kernels:
// device/k_fft.h, device/k_full.h.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ocean_internal.h"
#include "launch_common.h"
#include "device/fft.h"
#include "device/grid.h"
#include "device/k_fft.h"
#include "device/k_full.h"
#include "device/memory.h"

namespace oceanfft
{

template <int LOGN>
int lds_bytes_rows()
{
  using S = FftShape<LOGN>;
  return ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + RowCfg<LOGN>::LDS_BYTES;
}
template <int LOGN>
int lds_bytes_cols()
{
  using S = FftShape<LOGN>;
  return ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + ColCfg<LOGN>::LDS_BYTES;
}


// B == 1 (N = 16384: one 256-KiB column per CU) makes the blocked layout column-major, whose rows
// the row pass could only read 16 bytes at a time. This tiled transpose (64 x 64 texels through
// LDS, 1-KiB runs on both sides) turns inter[c][src][img][x_local][y] into row-major
// out[c][img][y][x] for the rank's w rows.
__global__ __launch_bounds__(256) void k_blocks_to_rows(int cascades, int n, int w, const float4* __restrict__ in,
                                                        float4* __restrict__ out)
{
  __shared__ float4 tile[64][65];
  const int tiles_x = n / 64, tiles_y = w / 64;
  const int total = cascades * 2 * tiles_x * tiles_y;
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    const int cimg = item / (tiles_x * tiles_y), t = item % (tiles_x * tiles_y);
    const int c = cimg >> 1, img = cimg & 1;
    const int tx = t % tiles_x, ty = t / tiles_x;
    // read: 64 columns x 64 rows; column x is contiguous in y
    for (int k = 0; k < 16; k++)
    {
      const int L = k * 256 + threadIdx.x, col = L >> 6, row = L & 63;
      const int x = tx * 64 + col, srcr = x / w, xl = x % w;
      tile[col][row] = in[(size_t)c * 2 * n * w + ((size_t)(srcr * 2 + img) * w + xl) * w + ty * 64 + row];
    }
    __syncthreads();
    for (int k = 0; k < 16; k++)
    {
      const int L = k * 256 + threadIdx.x, row = L >> 6, col = L & 63;
      out[((size_t)cimg * w + ty * 64 + row) * n + tx * 64 + col] = tile[col][row];
    }
    __syncthreads();
  }
}

hipError_t launch_cols_evolve(int logn, const FrameParams& fp, const SlabGeom& g, const float4* h0, float4* inter,
                              const float2* tw, hipStream_t stream, int cus, int keep)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    using K = ColFirstCfg<LOGN>;
    using S = FftShape<LOGN>;
    auto kern = keep >= 16 ? k_cols_evolve<LOGN, 16>
                           : (keep >= 8 ? k_cols_evolve<LOGN, 8> : (keep >= 4 ? k_cols_evolve<LOGN, 4> : k_cols_evolve<LOGN, 0>));
    const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + K::LDS1;
    const int items = fp.cascades * ((g.w / K::B) / K::SPW);
    const int grid = persistent_grid(kern, K::WG1, lds, items, cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG1), lds, stream, fp, g, h0, inter, tw);
    return hipGetLastError();
  });
}

bool ifft_fourstep_supported(int logn) { return fourstep_table(logn); }

size_t ifft_fourstep_work_texels(int logn, int wc) { return ((size_t)1 << logn) * (size_t)wc; }

// Rows in place, then per slab of wc columns: step 1 (images -> work slab), step 2 (slab -> images).
// Bytes: 3 x 32 per texel (the in-place order: 2 x 32, but its column pass reads and writes 16-B
// pieces at N = 16384). Measured (tools/microbench/ifft4bench, profiles/r02_ifft4bench.log), one
// 16384^2 image: in place 7.26 ms, four-step 5.05 ms (wc 2048); at 8192 the in-place order (two
// columns per item, 32-B pieces) stays ahead, 4.78 vs 4.96 ms for 4 images.

hipError_t launch_ifft_fourstep(int logn, int n_images, float4* images, float4* work, int wc, const float2* tw,
                                const float2* tw2, hipStream_t stream, int cus)
{
  if (!ifft_fourstep_supported(logn) || !tw2)
    return hipErrorInvalidValue;
  const int n = 1 << logn;
  if (wc < 64 || wc > n || n % wc != 0 || (wc & 63) != 0)
    return hipErrorInvalidValue;
  hipError_t e = launch_rows_ifft(logn, n_images, images, tw, stream, cus);
  if (e != hipSuccess)
    return e;
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (LOGN < 13)
      return hipErrorInvalidValue;
    else
    {
      constexpr int LOGN2 = LOGN - 4;
      using K2 = ColCfg<LOGN2>;
      auto k1 = k_cols4_step1<LOGN>;
      auto k2 = k_cols4_step2<LOGN2>;
      const int lds2 = lds_bytes_cols<LOGN2>();
      for (int im = 0; im < n_images; im++)
        for (int x0 = 0; x0 < n; x0 += wc)
        {
          float4* img = images + ((size_t)im << (2 * LOGN));
          const int g1 = persistent_grid(k1, 256, 0, (wc / 64) * ((n / 16) / 4), cus);
          hipLaunchKernelGGL(k1, dim3(g1), dim3(256), 0, stream, 1, x0, wc, img, work, tw);
          const int g2 = persistent_grid(k2, K2::WG, lds2, 16 * (wc / K2::C), cus);
          hipLaunchKernelGGL(k2, dim3(g2), dim3(K2::WG), lds2, stream, 1, x0, wc, work, img, tw2);
          const hipError_t le = hipGetLastError();
          if (le != hipSuccess)
            return le;
        }
      return hipSuccess;
    }
  });
}

// Column-first EncodeIFFT through a work image: 4096 (B = 4) and 8192 (B = 2: the strided pass only
// reads the 32-B pieces, which L2 merges, and writes whole strips; the in-place column pass wrote
// them back as partial lines, 1.67 x algorithmic). At 8192 a 128-B line of the work image holds 4
// rows = 2 row items, run as pairs on one XCD (GRPR 2): 4 x 8192^2 in 4.39 ms against 5.06 ungrouped
// and 4.77 in place (tools/microbench/ifft4bench, profiles/r03_ifft4bench.log).
bool ifft_colfirst_supported(int logn) { return logn == 12 || logn == 13; }

hipError_t launch_ifft_colfirst(int logn, int n_images, float4* images, float4* work, const float2* tw,
                                hipStream_t stream, int cus)
{
  if (!ifft_colfirst_supported(logn))
    return hipErrorInvalidValue;
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (LOGN != 12 && LOGN != 13)
      return hipErrorInvalidValue;
    else
    {
      using K = ColFirstCfg<LOGN>;
      using S = FftShape<LOGN>;
      constexpr int tw_lds = tw_bytes<S::TW_ENTRIES>();
      {
        auto kern = k_cols_to_blocks<LOGN>;
        const int lds = tw_lds + K::LDS1;
        const int grid = persistent_grid(kern, K::WG1, lds, n_images * (S::N / K::B), cus);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG1), lds, stream, n_images, images, work, tw);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess)
          return e;
      }
      // row items sharing one 128-B line (8 texels) of the work image: B x RPW texels per item each.
      // 4096: one row per 256-thread item (four workgroups per CU instead of one 4-row workgroup),
      // the two items of each line on one XCD with default-policy loads, as at 8192: 8 x 4096^2
      // 1.779 -> 1.697 ms (tools/microbench/prebench, profiles/r03_prebench_4096.log)
      constexpr int RPW = LOGN == 12 ? 1 : K::RPW2, LAR = LOGN == 12 ? 0 : kStream;
      constexpr int GRPR = K::B * RPW >= 8 ? 1 : 8 / (K::B * RPW);
      auto kern = k_rows_final<LOGN, true, LAR, kStream, RPW, 0, GRPR>;
      const int lds = tw_lds + lds_row_slots<LOGN>(RPW) * 8;
      const SlabGeom g{0, S::N};
      const int grid = persistent_grid(kern, S::T * RPW, lds, n_images * (S::N / RPW), cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(S::T * RPW), lds, stream, n_images, g, work, images, (float*)nullptr,
                         FoamParams{}, tw);
      return hipGetLastError();
    }
  });
}

// EncodeIFFT at N = 8192 / 16384 with the radix-R pre-stage column pass (k_cols_pre) through a work
// image, then the row pass. WL 0: blocked work, k_rows_final with the row permutation (GRPR row items
// sharing a 128-B line of the B = 4 blocks on one XCD: 1 at 8192, where an item reads 2 rows = whole
// lines, 2 at 16384); WL 1: row-major work, k_rows_ifft_out. twm: the 4096-point table.
template <int LOGN, int WL, int LA = 0, int LAR = kStream, int RPW = (LOGN == 13 ? 2 : 1), int LB = 2>
hipError_t launch_ifft_pre_t(int n_images, float4* images, float4* work, const float2* twn, const float2* twm,
                             hipStream_t stream, int cus)
{
  using S = FftShape<LOGN>;
  using P = PreCfg;
  constexpr int R = S::N / P::M;
  {
    auto kern = k_cols_pre<LOGN, LA, WL, LB>;  // 8 loads in flight per batch
    const int lds = P::TWM + tw_bytes<S::TW_ENTRIES>() + P::XCH;
    const int grid = persistent_grid(kern, P::WG, lds, n_images * (S::N / P::B) * R, cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(P::WG), lds, stream, n_images, images, work, twn, twm);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
      return e;
  }
  constexpr int tw_lds = tw_bytes<S::TW_ENTRIES>();
  if constexpr (WL == 0)
  {
    constexpr int GRPR = P::B * RPW >= 8 ? 1 : 8 / (P::B * RPW);
    auto kern = k_rows_final<LOGN, true, LAR, kStream, RPW, 0, GRPR, P::B, R>;
    const int lds = tw_lds + lds_row_slots<LOGN>(RPW) * 8;
    const SlabGeom g{0, S::N};
    const int grid = persistent_grid(kern, S::T * RPW, lds, n_images * (S::N / RPW), cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(S::T * RPW), lds, stream, n_images, g, work, images, (float*)nullptr,
                       FoamParams{}, twn);
  }
  else
  {
    using RC = RowCfg<LOGN>;
    auto kern = k_rows_ifft_out<LOGN>;
    const int lds = tw_lds + RC::LDS_BYTES;
    const int grid = persistent_grid(kern, RC::WG, lds, n_images << LOGN, cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(RC::WG), lds, stream, n_images << LOGN, (const float4*)work, images,
                       twn);
  }
  return hipGetLastError();
}

bool ifft_pre_supported(int logn) { return logn == 13; }

hipError_t launch_ifft_pre(int logn, int n_images, float4* images, float4* work, const float2* twn, const float2* twm,
                           hipStream_t stream, int cus)
{
  // 8192: one-row row items (512 threads, two workgroups per CU), the two items of each 128-B line
  // on one XCD with default-policy loads so the partner's half is an L2 hit. 2 x 8192^2 (prebench,
  // profiles/r03_prebench.log): 2.231 ms (production column-first) -> 1.860 ms; the two-row items
  // 2.043, streamed row loads 1.975, row-major work 2.104. At 16384 the R = 4 pass (6.1 ms for 2
  // images: each item reads its strip 4 times, 48 us per item) plus the blocked row pass (4.6 ms)
  // lose to the four-step order (9.7 vs 10.6 ms): not used there.
  if (logn == 13)
    return launch_ifft_pre_t<13, 0, 0, 0, 1>(n_images, images, work, twn, twm, stream, cus);
  return hipErrorInvalidValue;
}

hipError_t launch_rows_final(int logn, int cascades, const SlabGeom& g, const float4* inter, float4* scratch,
                             float4* maps, float* jac, const FoamParams& foam, const float2* tw, hipStream_t stream,
                             int cus)
{
  const bool transpose = rows_need_transpose(logn) && scratch != nullptr;
  if (transpose)
  {
    const int n = 1 << logn;
    const int items = cascades * 2 * (n / 64) * (g.w / 64);
    const int grid = persistent_grid(k_blocks_to_rows, 256, 0, items, cus);
    hipLaunchKernelGGL(k_blocks_to_rows, dim3(grid), dim3(256), 0, stream, cascades, n, g.w, inter, scratch);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
      return e;
  }
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    using K = ColFirstCfg<LOGN>;
    using S = FftShape<LOGN>;
    const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + K::LDS2;
    const int items = cascades * 2 * (g.w / K::RPW2);
    if (transpose)
    {
      auto kern = k_rows_final<LOGN, false>;
      const int grid = persistent_grid(kern, K::WG2, lds, items, cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG2), lds, stream, 2 * cascades, g, scratch, maps, jac, foam, tw);
    }
    else
    {
      // B x RPW2 texels per item and strip; items sharing a 128-B line run together on one XCD (8192)
      constexpr int GRPR = K::B * K::RPW2 >= 8 ? 1 : 8 / (K::B * K::RPW2);
      auto kern = k_rows_final<LOGN, true, kStream, kStream, K::RPW2, 0, GRPR>;
      const int grid = persistent_grid(kern, K::WG2, lds, items, cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG2), lds, stream, 2 * cascades, g, inter, maps, jac, foam, tw);
    }
    return hipGetLastError();
  });
}

hipError_t launch_rows_ifft_rows(int logn, int rows, float4* data, const float2* tw, hipStream_t stream, int cus)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    using R = RowCfg<LOGN>;
    auto kern = k_rows_ifft<LOGN>;
    int lds = lds_bytes_rows<LOGN>();
    int items = (rows + R::RPW - 1) / R::RPW;
    int grid = persistent_grid(kern, R::WG, lds, items, cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(R::WG), lds, stream, rows, data, tw);
    return hipGetLastError();
  });
}

hipError_t launch_rows_ifft(int logn, int n_images, float4* images, const float2* tw, hipStream_t stream, int cus)
{
  return launch_rows_ifft_rows(logn, n_images << logn, images, tw, stream, cus);
}

hipError_t launch_cols(int logn, int n_images, float4* images, const float2* tw, hipStream_t stream, int cus)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    using K = ColCfg<LOGN>;
    using S = FftShape<LOGN>;
    int lds = lds_bytes_cols<LOGN>();
    int items = n_images * K::STRIPS;
    if constexpr (K::C > 4 && LOGN >= 8)
      if (items < cus)
      {
        // fewer 16-column strips than CUs (one 1024^2 image: 64): 4-column strips, 256-thread
        // workgroups; a strip pair's 64-B row pieces meet in one L2 (GROUP 2)
        constexpr int CC = 4;
        auto narrow = k_cols<LOGN, 2, CC>;
        const int ldsn = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + CC * S::PADDED * 8;
        const int grid = persistent_grid(narrow, S::T * CC, ldsn, n_images * (S::N / CC), cus);
        hipLaunchKernelGGL(narrow, dim3(grid), dim3(S::T * CC), ldsn, stream, n_images, images, tw);
        return hipGetLastError();
      }
    auto kern = k_cols<LOGN>;
    int grid = persistent_grid(kern, K::WG, lds, items, cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG), lds, stream, n_images, images, tw);
    return hipGetLastError();
  });
}

}  // namespace oceanfft
