// launch_slab.hip — the half-spectrum frame of slabs (one grid over P ranks) and of
// whole grids of 8192 / 16384: the four-step column pass writing destination-block order (default
// at 8192 / 16384) and the strip-dealt column pass + transposes (slabs of 1024 .. 4096, and
// ocean_generator_set_four_step(0)). Kernels: device/k_gen4.h, device/k_half_cols.h,
// device/k_half_rows.h.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ocean_internal.h"
#include "launch_common.h"
#include "device/grid.h"
#include "device/k_gen4.h"
#include "device/k_half_cols.h"
#include "device/k_half_rows.h"
#include "device/k_rows_hp.h"
#include "device/k_rows_xs.h"
#include "device/spectrum.h"

namespace oceanfft
{

// ---- strip-dealt half-spectrum path (slabs, and whole grids of N = 8192 / 16384) ----
bool half_slab_supported(int logn) { return logn >= 10 && logn <= 14; }

int half_strips(int logn) { return (1 << logn) / (2 * spectrum_block(logn)) + 1; }

// block = gab | gde | gc parts (40 B per element) | the Nyquist-row term [c][2][N] float4
static size_t half_slab_spec_offset(int logn, int cascades, const HalfSlab& h)
{
  return (size_t)40 * cascades * h.S * h.w * spectrum_block(logn);
}

size_t half_slab_block_bytes(int logn, int cascades, const HalfSlab& h)
{
  return half_slab_spec_offset(logn, cascades, h) + (size_t)cascades * 2 * (1 << logn) * sizeof(float4);
}

size_t half_slab_row_texels(int logn, int cascades, int w)
{
  return (size_t)cascades * w * half_strips(logn) * spectrum_block(logn);
}

hipError_t launch_half_slab_columns(int logn, const FrameParams& fp, const HalfSlab& hsl, int ranks, const float4* h0,
                                    bool h0_full, const float4* h0row, void* send, const float2* tw,
                                    hipStream_t stream, int cus, float2* hs, int hs_blocks, const Gen4Put* put)
{
  if (put && (!put->dst || (put->stream && put->stream != stream)))
    return hipErrorInvalidValue;
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (!HalfCfg<LOGN>::SLAB_SUPPORTED)
      return hipErrorInvalidValue;
    else
    {
      using K = ColFirstCfg<LOGN>;
      using S = FftShape<LOGN>;
      const int n = S::N;
      if (hsl.w % S::T != 0 || !hs)
        return hipErrorInvalidValue;
      const size_t blk = half_slab_block_bytes(LOGN, fp.cascades, hsl);
      hipError_t e = hipSuccess;
      // the one-sided exchange stores into the peers' receive slots: only once they are free
      if (put && put->start)
        e = hipEventRecord(put->start, stream);
      if (e == hipSuccess && put && put->wait)
        e = launch_peer_wait(*put->wait, stream);
      if (e != hipSuccess)
        return e;
      const int cus2 = put && put->cus > 0 ? put->cus : cus;
      const size_t spec_off = half_slab_spec_offset(LOGN, fp.cascades, hsl);
      e = put ? launch_half_nyquist(fp, n, K::B, h0, nullptr, h0_full ? nullptr : h0row, ranks, 0, nullptr, stream, cus2,
                                    put->dst, spec_off)
              : launch_half_nyquist(fp, n, K::B, h0, reinterpret_cast<float4*>((unsigned char*)send + spec_off),
                                    h0_full ? nullptr : h0row, ranks, blk, nullptr, stream, cus);
      if (e != hipSuccess || hsl.nstrips < 1)  // a rank past the last strip only builds the Nyquist-row term
        return e;
      // slab items keep fewer pairs in VGPRs: with four, the SLAB store addressing spills 8-16 B (at
      // N = 8192 already with two; one fits)
      constexpr int HKS = LOGN == 13 ? 1 : kHalfHK - 1;
      auto kern = put ? k_cols_half<LOGN, kStream, kStream, true, true, false, 1, 1, K::B, true, false, kHalfHL, HKS, 0, 4, true>
                      : k_cols_half<LOGN, kStream, kStream, true, true, false, 1, 1, K::B, true, false, kHalfHL, HKS>;
      const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + K::LDS1 + kHalfHL * K::WG1 * 16;
      int grid = persistent_grid(kern, K::WG1, lds, fp.cascades * hsl.nstrips, cus2);
      if (grid > hs_blocks)
        grid = hs_blocks;
      unsigned char* target = put ? reinterpret_cast<unsigned char*>(const_cast<uint64_t*>(put->dst))
                                  : static_cast<unsigned char*>(send);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG1), lds, stream, fp, h0, (float4*)nullptr, (float4*)nullptr,
                         (float2*)nullptr, tw, hs, hsl, target, h0_full ? 1 : 0, (const SpectrumConsts*)nullptr);
      return hipGetLastError();
    }
  });
}

// The row pass over row-major fields (RowSrc: the strip-dealt path's one block after k_half_to_rows,
// or the four-step path's exchange blocks). N = 16384 (T = 1024, one row per workgroup): the XS x
// transform (barriers 14 -> 7 per image), which needs tw2, the N/16-point table ocean_fft_create
// appends for the sizes fourstep_table() names.
// tools/microbench A/B at 16384: 0 = the plain transform, 1 = XS (k_rows_half), 2 = k_rows_xs, 3 =
// k_rows_xs with 2 of the next image's 8 field loads in flight during the transform (PF; 4 spill), 4 =
// k_rows_xs EARLY 4 on a resident grid: every image's loads issued before the previous image's stores,
// and image 0's C kept for image 1 (round 5: 3.677 -> 3.158 (EARLY 3) -> 3.076 ms per 16384^2 pass,
// maps bit-identical, profiles/r05_rm16bench_early.log, r05_rm16bench_keepc.log).
// Measured and not kept: k_rows_xp (tools/microbench/k_rows_xp.h, the 64 x 256 split with the
// sub-transforms' exchanges in the wave), 3.80-3.83 against 3.74 ms (profiles/r04_rm16bench_xp.log).
inline int rm_rows_variant = 4;

template <int LOGN>
hipError_t launch_rm_rows(const FrameParams& fp, const RowSrc& rs, const float4* spec, float4* maps, float* jac,
                          const FoamParams& foam, const float2* tw, const float2* tw2, int rows, hipStream_t stream,
                          int cus)
{
  using S = FftShape<LOGN>;
  constexpr int RPW = S::T >= 1024 ? 1 : 2;
  // the block index of a wave's loads must be wave-uniform, and is taken with a shift
  if (rs.cpr < 64 || (rs.cpr & (rs.cpr - 1)) != 0 || rows % RPW != 0)
    return hipErrorInvalidValue;
  if constexpr (LOGN == 12)
  {
    // the strip-dealt slabs at 4096: the whole grid's row pass (k_rows_hp, launch_half_rows) on
    // row-major fields, so slab frames stay bit-identical to whole grids
    if (half_rows_variant == 1)
    {
      auto kern = k_rows_hp<1, 1, true>;
      const int grid = persistent_grid(kern, 256, HpCfg::LDS, fp.cascades * rows, cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), HpCfg::LDS, stream, fp, (const float4*)nullptr,
                         (const float4*)nullptr, (const float2*)nullptr, spec, maps, jac, foam, tw, rows, rs);
      return hipGetLastError();
    }
  }
  if constexpr (RPW == 1)
  {
    if (rm_rows_variant >= 2)
    {
      if (!tw2)
        return hipErrorInvalidValue;
      auto kern = rm_rows_variant == 4 ? k_rows_xs<LOGN, 0, 4> : rm_rows_variant == 3 ? k_rows_xs<LOGN, 2> : k_rows_xs<LOGN, 0>;
      const int lds = XsCfg<LOGN>::LDS;
      const int grid = rm_rows_variant == 4 ? resident_grid(kern, S::T, lds, fp.cascades * rows, cus)
                                            : persistent_grid(kern, S::T, lds, fp.cascades * rows, cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(S::T), lds, stream, fp, spec, maps, jac, foam, tw, rows, rs, tw2);
      return hipGetLastError();
    }
    if (rm_rows_variant != 0)
    {
      if (!tw2)
        return hipErrorInvalidValue;
      auto kern = k_rows_half<LOGN, kStream, kStream, 0, 1, true, true, 1, 1, 4, 2, true, true>;
      const int lds = XsCfg<LOGN>::LDS;
      const int grid = persistent_grid(kern, S::T, lds, fp.cascades * rows, cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(S::T), lds, stream, fp, (const float4*)nullptr, (const float4*)nullptr,
                         (const float2*)nullptr, spec, maps, jac, foam, tw, rows, rs, tw2);
      return hipGetLastError();
    }
  }
  auto kern = k_rows_half<LOGN, kStream, kStream, 0, RPW, true, true>;
  const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + lds_row_slots<LOGN>(RPW) * 8;
  const int grid = persistent_grid(kern, S::T * RPW, lds, fp.cascades * (rows / RPW), cus);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(S::T * RPW), lds, stream, fp, (const float4*)nullptr, (const float4*)nullptr,
                     (const float2*)nullptr, spec, maps, jac, foam, tw, rows, rs, (const float2*)nullptr);
  return hipGetLastError();
}

hipError_t launch_half_slab_rows(int logn, const FrameParams& fp, const HalfSlab& hsl, const void* recv, float4* rm_ab,
                                 float4* rm_de, float2* rm_c, float4* maps, float* jac, const FoamParams& foam,
                                 const float2* tw, const float2* tw2, hipStream_t stream, int cus)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (!HalfCfg<LOGN>::SLAB_SUPPORTED)
      return hipErrorInvalidValue;
    else
    {
      using S = FftShape<LOGN>;
      const int n = S::N, B = spectrum_block(LOGN), C = fp.cascades;
      if (hsl.w % kHalfToRowsTY != 0)
        return hipErrorInvalidValue;
      const size_t part = (size_t)C * hsl.S * hsl.w * B, blk = half_slab_block_bytes(LOGN, C, hsl);
      const float4* spec = reinterpret_cast<const float4*>((const unsigned char*)recv +
                                                           half_slab_spec_offset(LOGN, C, hsl));  // block 0's copy
      const int kp = half_strips(LOGN) * B;
      const int tiles = C * ((half_strips(LOGN) + hsl.S - 1) / hsl.S) *
                        ((hsl.S * B + kHalfToRowsTU - 1) / kHalfToRowsTU) * (hsl.w / kHalfToRowsTY);
      const int tgrid = (one_shot_grids(cus) || tiles < cus * 4) ? tiles : cus * 4;
      const unsigned char* in = (const unsigned char*)recv;
      constexpr int KB = ColFirstCfg<LOGN>::B;
      hipLaunchKernelGGL((k_half_to_rows<float4, KB>), dim3(tgrid), dim3(256), 0, stream, C, n, hsl, in, (size_t)0, blk, rm_ab);
      hipLaunchKernelGGL((k_half_to_rows<float4, KB>), dim3(tgrid), dim3(256), 0, stream, C, n, hsl, in, part * 16, blk, rm_de);
      hipLaunchKernelGGL((k_half_to_rows<float2, KB>), dim3(tgrid), dim3(256), 0, stream, C, n, hsl, in, part * 32, blk, rm_c);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess)
        return e;
      const RowSrc rs{reinterpret_cast<const unsigned char*>(rm_ab), reinterpret_cast<const unsigned char*>(rm_de),
                      reinterpret_cast<const unsigned char*>(rm_c), 0, n / 2, kp, 0};
      return launch_rm_rows<LOGN>(fp, rs, spec, maps, jac, foam, tw, tw2, hsl.w, stream, cus);
    }
  });
}

// ---- the four-step column pass (N = 8192 / 16384): whole grids and slabs (device/k_gen4.h) ----
// the four-step paths read the N/16-point table ocean_fft_create appends under the same predicate
bool gen4_supported(int logn) { return fourstep_table(logn); }

int gen4_h0_block() { return kGen4Block; }

Gen4Geom gen4_geom(int logn, int cascades, int rank, int ranks, bool whole_h0)
{
  const int n = 1 << logn;
  Gen4Geom g{};
  g.ranks = ranks;
  g.w = n / ranks;
  g.cols = n / (2 * ranks);
  g.u0 = rank * g.cols;
  g.nyq = rank == ranks - 1 ? 1 : 0;
  g.lp = g.cols + 16;  // whole 128-B lines per row for both element sizes (cols % 64 == 0)
  if (whole_h0)
  {
    // the whole grid's h0 image, blocked kGen4Block columns wide over x: column x = N/2 + u' is in
    // block (N/2 + u') / 64, and x = 0 starts block 0
    g.h0_cstride = (size_t)n * n;
    g.h0_reg = (size_t)(n / 2) * n;
    g.h0_nyq = 0;
  }
  else
  {
    // the rank's own columns, blocked from its first one, then (rank P - 1) the block of x = 0 .. 63
    const size_t xb = (size_t)g.cols / kGen4Block + g.nyq;
    g.h0_cstride = xb * n * kGen4Block;
    g.h0_reg = 0;
    g.h0_nyq = (size_t)(g.cols / kGen4Block) * n * kGen4Block;
  }
  g.blk_bytes = (size_t)40 * cascades * g.w * g.lp + (size_t)cascades * 2 * n * sizeof(float4);
  return g;
}

size_t gen4_parts_bytes(int logn, int cascades, const Gen4Geom& g)
{
  return (size_t)40 * cascades * ((size_t)1 << logn) * g.lp;
}

// byte offsets of the fields inside an exchange block: gab | gde | gc | the Nyquist-row term
static size_t gen4_part_offset(int cascades, const Gen4Geom& g, int part)
{
  const size_t t = (size_t)cascades * g.w * g.lp;
  return part == 0 ? 0 : part == 1 ? 16 * t : part == 2 ? 32 * t : 40 * t;
}

hipError_t launch_gen4_columns(int logn, const FrameParams& fp, const Gen4Geom& g, const float4* h0, const float4* h0row,
                               void* parts, void* send, const float2* tw, const float2* tw2, hipStream_t stream, int cus,
                               const Gen4Put* put)
{
  if (!tw2 || g.cols % kGen4Block != 0 || (put && !put->dst))
    return hipErrorInvalidValue;
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (LOGN < 13)
      return hipErrorInvalidValue;
    else
    {
      constexpr int N = 1 << LOGN, N2 = N / 16, LOGN2 = LOGN - 4;
      const int C = fp.cascades;
      unsigned char* snd = static_cast<unsigned char*>(send);
      // step 1: h0 -> the rank's parts [c][N][lp]
      auto k1 = k_gen4_step1<LOGN>;
      const int ncols = g.cols + g.nyq;
      const int items = C * ((ncols + 63) / 64) * (N2 / 4);
      hipLaunchKernelGGL(k1, dim3(persistent_grid(k1, 256, 0, items, cus)), dim3(256), 0, stream, fp, g, h0,
                         (unsigned char*)parts, tw);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess)
        return e;
      // the put on its own stream (pipelined one-sided frames): after step 1
      if (put && put->stream && put->stream != stream)
      {
        if (!put->handoff)
          return hipErrorInvalidValue;
        e = hipEventRecord(put->handoff, stream);
        if (e == hipSuccess)
          e = hipStreamWaitEvent(put->stream, put->handoff, 0);
        if (e != hipSuccess)
          return e;
        stream = put->stream;
      }
      // the one-sided exchange writes into the peers' receive slots: only once they are free
      if (put && put->start)
      {
        e = hipEventRecord(put->start, stream);
        if (e != hipSuccess)
          return e;
      }
      if (put && put->wait)
      {
        e = launch_peer_wait(*put->wait, stream);
        if (e != hipSuccess)
          return e;
      }
      const int cus2 = put && put->cus > 0 ? put->cus : cus;
      // the Nyquist-row term, into every destination block (each frame's row pass reads its own)
      e = put ? launch_half_nyquist(fp, N, kGen4Block, h0, nullptr, h0row, g.ranks, 0, nullptr, stream, cus2, put->dst,
                                    gen4_part_offset(C, g, 3))
              : launch_half_nyquist(fp, N, kGen4Block, h0, reinterpret_cast<float4*>(snd + gen4_part_offset(C, g, 3)),
                                    h0row, g.ranks, g.blk_bytes, nullptr, stream, cus);
      if (e != hipSuccess)
        return e;
      // step 2: parts -> destination blocks. 8 columns per workgroup at N2 = 1024 (512 threads, two per
      // CU: 2.145 -> 2.015 ms for the three parts at 16384, tools/microbench/gen4bench); ColCfg's 16 at
      // N2 = 512 (already 512 threads)
      constexpr int CI = ColCfg<LOGN2>::C * FftShape<LOGN2>::T >= 1024 ? ColCfg<LOGN2>::C / 2 : ColCfg<LOGN2>::C;
      constexpr int WG2 = FftShape<LOGN2>::T * CI;
      const size_t part = (size_t)C * N * g.lp;  // texels per part
      const float4* wab = static_cast<const float4*>(parts);
      const float4* wde = wab + part;
      const float4* wc = wde + part;  // gc (float2 texels) viewed as pairs of columns
      const int lds2 = ((FftShape<LOGN2>::TW_ENTRIES * 8 + 15) / 16) * 16 + CI * FftShape<LOGN2>::PADDED * 8;
      auto sp = put ? k_gen4_step2<LOGN2, true, CI, true> : k_gen4_step2<LOGN2, true, CI>;
      auto sc = put ? k_gen4_step2<LOGN2, false, CI, true> : k_gen4_step2<LOGN2, false, CI>;
      const uint64_t* dst = put ? put->dst : nullptr;
      const int pcols = (ncols + 1) / 2;
      const int gp = persistent_grid(sp, WG2, lds2, C * 16 * ((ncols + CI - 1) / CI), cus2);
      const int gcg = persistent_grid(sc, WG2, lds2, C * 16 * ((pcols + CI - 1) / CI), cus2);
      hipLaunchKernelGGL(sp, dim3(gp), dim3(WG2), lds2, stream, C, ncols, g.lp, wab, snd, gen4_part_offset(C, g, 0), g, tw2,
                         dst);
      hipLaunchKernelGGL(sp, dim3(gp), dim3(WG2), lds2, stream, C, ncols, g.lp, wde, snd, gen4_part_offset(C, g, 1), g, tw2,
                         dst);
      hipLaunchKernelGGL(sc, dim3(gcg), dim3(WG2), lds2, stream, C, pcols, g.lp / 2, wc, snd, gen4_part_offset(C, g, 2), g,
                         tw2, dst);
      return hipGetLastError();
    }
  });
}

hipError_t launch_gen4_rows(int logn, const FrameParams& fp, const Gen4Geom& g, const void* recv, float4* maps, float* jac,
                            const FoamParams& foam, const float2* tw, const float2* tw2, hipStream_t stream, int cus)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (LOGN < 13)
      return hipErrorInvalidValue;
    else
    {
      const int C = fp.cascades;
      const unsigned char* r = static_cast<const unsigned char*>(recv);
      // row y's columns: P runs of `cols` texels, one per source block; Nyquist column in block P - 1
      const RowSrc rs{r + gen4_part_offset(C, g, 0), r + gen4_part_offset(C, g, 1), r + gen4_part_offset(C, g, 2),
                      g.blk_bytes, g.cols, g.lp, g.ranks - 1};
      const float4* spec = reinterpret_cast<const float4*>(r + gen4_part_offset(C, g, 3));  // block 0's copy
      return launch_rm_rows<LOGN>(fp, rs, spec, maps, jac, foam, tw, tw2, g.w, stream, cus);
    }
  });
}

}  // namespace oceanfft
