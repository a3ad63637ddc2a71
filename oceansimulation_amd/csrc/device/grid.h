// device/grid.h — work placement and the shared pass geometry: the XCD-aware block -> item maps,
// the column-first pass configuration (ColFirstCfg) and the in-place column pass's (ColCfg), and the
// cache-policy constant of streamed accesses.
#pragma once

#include <hip/hip_runtime.h>

#include "device/fft.h"

namespace oceanfft
{

// Block -> work-slot map that gives blocks b and b+8 (same XCD under round-robin placement)
// adjacent strips, so both 64-B halves of a 128-B line meet in one L2. Speed only; any placement
// is correct.
// Generalisation: GROUP consecutive work slots on blocks b, b+8, ..., b+8(GROUP-1) (one XCD).
template <int GROUP>
__device__ __forceinline__ int xcd_group_slot(int b, int G)
{
  if (G % (8 * GROUP) != 0)
    return b;
  const int xcd = b & 7, j = b >> 3;
  const int grp = xcd * (G / (8 * GROUP)) + j / GROUP;
  return GROUP * grp + j % GROUP;
}

__device__ __forceinline__ int xcd_pair_slot(int b, int G)
{
  if ((G & 15) != 0)
    return b;
  int xcd = b & 7, j = b >> 3;
  int pair = xcd * (G >> 4) + (j >> 1);
  return 2 * pair + (j & 1);
}

// ------------------------------------------------------------------------------------------------
// Generator path, column-first (2 HBM passes, every global access a >= 256-byte run per wave):
//   h0      [cascade][xb][y][B]                 strip-blocked (written by k_generate_spectrum)
//   pass 1  k_cols_evolve: per strip of B columns: evolve (spectrum.compute:183-240), iFFT along y
//           of both packed images, write inter[cascade][img][xb][y][B] (contiguous runs)
//   pass 2  k_rows_final: per RPW2 rows of one image: read the blocked intermediate (lanes
//           interleaved so 8 lanes cover one 256-byte run of B texels x RPW2 rows), iFFT along x,
//           write the row-major map (the reference's RGBA32F image) and, for displacement maps,
//           the Jacobian (spectrum.compute:246-259).
// The reference transforms rows first (src/FFTCalculator.cpp:19-20); the 2D iFFT is separable, so
// the order changes only rounding (covered by the parity tolerance).
// ------------------------------------------------------------------------------------------------
template <int LOGN>
struct ColFirstCfg
{
  using S = FftShape<LOGN>;
  static constexpr int N = S::N, T = S::T;
  static constexpr int B = T >= 1024 ? 1 : (T >= 512 ? 2 : (T < 4 ? T : 4));  // texels per block row
  // Below N = 1024 (the full-spectrum path: the reference's own 256^2 cascades) an item is one wave's
  // worth of strips / rows (64 threads) instead of four waves' (round 6: a 3 x 256^2 frame had 48 column
  // and 96 row workgroups for 256 CUs); the per-column arithmetic is the same.
  static constexpr int SPW_RAW = T >= 64 ? (256 / (T * B) < 1 ? 1 : 256 / (T * B)) : (64 / (T * B) < 1 ? 1 : 64 / (T * B));
  static constexpr int SPW = SPW_RAW > N / B ? N / B : SPW_RAW;  // strips per pass-1 item
  static constexpr int C1 = B * SPW;                              // columns per pass-1 item
  static constexpr int WG1 = T * C1;
  static constexpr int LDS1 = C1 * S::PADDED * 8;  // float2 (split-lane) exchange
  static constexpr int RPW2_RAW = T < 64 ? 64 / T : (256 / T >= 4 ? 256 / T : (1024 / T < 4 ? 1024 / T : 4));
  static constexpr int RPW2 = RPW2_RAW > N ? N : RPW2_RAW;  // rows per pass-2 item
  static constexpr int WG2 = T * RPW2;
  static constexpr int LDS2 = lds_row_slots<LOGN>(RPW2) * 8;
};

// Cache policy: data touched once per frame (the KEEP once-read h0 texels, every store) is
// streamed non-temporally (LA, SA = kStream: 3-5 % faster per pass than the default policy); the
// twice-read h0 texels use the default policy (LR = 0) so the second read hits the cache
// hierarchy instead of HBM (6 % faster pass 1 than streaming them; tools/microbench/genbench).
constexpr int kStream = 2;

// ------------------------------------------------------------------------------------------------
// In-place column pass of the standalone EncodeIFFT: strips of C texel columns, transformed along y.
// ------------------------------------------------------------------------------------------------
template <int LOGN>
struct ColCfg
{
  using S = FftShape<LOGN>;
  static constexpr int C = S::T >= 1024 ? 1 : (1024 / S::T > 16 ? 16 : 1024 / S::T);
  static constexpr int WG = S::T * C;
  static constexpr int LDS_BYTES = C * S::PADDED * 8;  // float2 (SPLIT) exchange
  static constexpr int STRIPS = S::N / C;
};

}  // namespace oceanfft
