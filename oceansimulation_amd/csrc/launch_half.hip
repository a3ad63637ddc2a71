// launch_half.hip — the half-spectrum generator frame of whole grids, N = 1024 .. 4096 (84 B per
// point): k_cols_half (evolve + y iFFT of the five field multiples of H over the kept
// columns) and k_rows_half (Hermitian rebuild + x iFFT + maps + Jacobian). Kernels:
// device/k_half_cols.h, device/k_half_rows.h. The A/B variants measured against these live in
// tools/microbench/ab_kernels.h, outside the library.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "oceanfft.h"
#include "ocean_internal.h"
#include "launch_common.h"
#include "device/grid.h"
#include "device/k_half_cols.h"
#include "device/k_half_rows.h"
#include "device/k_rows_hp.h"
#include "device/spectrum.h"

namespace oceanfft
{

bool half_spectrum_supported(int logn) { return logn >= 10 && logn <= 12; }

int half_h0_block(int logn, int cascades) { return half_fields_fb(logn, cascades) == 2 ? 2 : spectrum_block(logn); }

// What launch_half_columns writes (and the h0 strips it reads): half strips into FB = 2 fields at 4096
// with <= 2 cascades, else whole strips into the production row groups.
HalfFieldLayout half_cols_layout(int logn, int cascades)
{
  if (half_fields_fb(logn, cascades) == 2)
    return {2, kHalfRG2, kHalfRGC2, 2};
  return {4, kHalfRG, kHalfRGC, spectrum_block(logn)};
}

// What launch_half_rows reads, per row-pass variant (1 = k_rows_hp at 4096, else k_rows_half).
HalfFieldLayout half_rows_layout(int logn, int cascades, int variant)
{
  const int hb = spectrum_block(logn);  // not read by the row pass: reported as the whole-strip width
  if (logn == 12 && variant == 1)
    return half_fields_fb(logn, cascades) == 2 ? HalfFieldLayout{2, kHalfRG2, kHalfRGC2, 2} : HalfFieldLayout{4, kHalfRG, kHalfRGC, hb};
  if (half_fields_fb(logn, cascades) == 2)
    return {2, kHalfRG2, kHalfRGC2, 2};
  return {4, kHalfRG, kHalfRGC, hb};
}

size_t half_field_texels(int logn)
{
  const size_t n = (size_t)1 << logn;
  return (n / 8 + 1) * n * 4;  // HalfCfg: STRIPS * N * B per cascade (B = 4)
}

size_t half_hs_bytes(int logn, int blocks)
{
  return half_slab_supported(logn) ? (size_t)blocks * 16 * 1024 * sizeof(float2) : 0;  // WG1 <= 1024
}

hipError_t launch_half_columns(int logn, const FrameParams& fp, const float4* h0, float4* gab, float4* gcd, float2* ge,
                               float4* spec, const float2* tw, hipStream_t stream, int cus, float2* hs, int hs_blocks,
                               const void* seed_consts, int h0_blk)
{
  if (!hs)  // the H scratch (half_hs_bytes): H evolved once per item instead of once per field round
    return hipErrorInvalidValue;
  const SpectrumConsts* seed = static_cast<const SpectrumConsts*>(seed_consts);
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (!HalfCfg<LOGN>::SUPPORTED)
      return hipErrorInvalidValue;
    else
    {
      using K = ColFirstCfg<LOGN>;
      using S = FftShape<LOGN>;
      const int hb = h0_blk > 0 ? h0_blk : K::B;
      if (hb != K::B && (hb != 2 || half_fields_fb(LOGN, fp.cascades) != 2))
        return hipErrorInvalidValue;  // 2-column h0 strips are read by the half-strip pass only
      // the Nyquist-row term (one row spectrum per image) is written by pass 1 itself (k_cols_half NYQ:
      // its least-loaded workgroup, after its items), into `spec` passed as the kernel's `send`
      // Field layout: row groups (kHalfRG, kHalfRGC). The H scratch in 16-B pairs (HP), one pair per
      // thread in the LDS the exchange leaves free (kHalfHL) and kHalfHK pairs in VGPRs at 4096 (2
      // below: 128 VGPRs, so two (2048) or four (1024) workgroups share a CU). h0 is read once per
      // item, streamed (nt), which leaves the XCD's L2 to the scratch. The fused re-seed frame (seed)
      // evaluates h0 in round 0 and keeps kHalfHKSeed pairs in VGPRs.
      constexpr int RG = kHalfRG, RGC = kHalfRGC;
      constexpr int HKW = LOGN == 12 ? kHalfHK : 2;
      const HalfFieldLayout lay = half_cols_layout(LOGN, fp.cascades);
      if constexpr (LOGN == 12 || LOGN == 11)
      {
        if (lay.fb == 2)
        {
          if (lay.rg != kHalfRG2 || lay.rgc != kHalfRGC2)
            return hipErrorInvalidValue;  // the kernels below are instantiated for this layout only
          // half strips (FB = 2): 2T-thread workgroups (512 at 4096, two per CU with a 68-KiB exchange
          // each; 256 at 2048, up to four per CU, two H pairs in VGPRs: with four, 8 B of spills)
          // h0 in 2-column strips (hb = 2, half_h0_block): each item streams its own strip
          constexpr int WGH = S::T * 2, HKH = LOGN == 12 ? kHalfHK : 2;
          auto kern = seed ? k_cols_half<LOGN, 0, kStream, true, false, true, kHalfRG2, kHalfRGC2, 2, true, false, kHalfHL,
                                         kHalfHKSeed, 0, 2, false, K::B, 0, true>
                           : k_cols_half<LOGN, kStream, kStream, true, false, false, kHalfRG2, kHalfRGC2, 2, true, false,
                                         kHalfHL, HKH, 0, 2, false, K::B, 0, true>;
          if (!seed && hb == 2)
            kern = k_cols_half<LOGN, kStream, kStream, true, false, false, kHalfRG2, kHalfRGC2, 2, true, false, kHalfHL,
                               HKH, 0, 2, false, 2, 0, true>;
          const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + 2 * S::PADDED * 8 + kHalfHL * WGH * 16;
          int grid = persistent_grid(kern, WGH, lds, fp.cascades * HalfCfg<LOGN>::STRIPS * 2, cus);
          const int slices = hs_blocks * (1024 / WGH);
          if (grid > slices)
            grid = slices;
          if (grid < 1)
            return hipErrorInvalidValue;
          hipLaunchKernelGGL(kern, dim3(grid), dim3(WGH), lds, stream, fp, h0, gab, gcd, ge, tw, hs, HalfSlab{},
                             reinterpret_cast<unsigned char*>(spec), 1, seed);
          return hipGetLastError();
        }
      }
      if (lay.fb != 4 || lay.rg != RG || lay.rgc != RGC || lay.h0_blk != K::B)
        return hipErrorInvalidValue;
      auto kern = seed ? k_cols_half<LOGN, 0, kStream, true, false, true, RG, RGC, K::B, true, false, kHalfHL, kHalfHKSeed,
                                     0, 4, false, K::B, 0, true>
                       : k_cols_half<LOGN, kStream, kStream, true, false, false, RG, RGC, K::B, true, false, kHalfHL, HKW, 0, 4,
                                     false, K::B, 0, true>;
      const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + K::LDS1 + kHalfHL * K::WG1 * 16;
      int grid = persistent_grid(kern, K::WG1, lds, fp.cascades * HalfCfg<LOGN>::STRIPS, cus);
      // hs holds hs_blocks slices for 1024-thread workgroups (half_hs_bytes); a block uses 16 x WG1
      // entries, so below 4096 each slice serves 1024 / WG1 blocks
      const int slices = hs_blocks * (1024 / K::WG1);
      if (grid > slices)
        grid = slices;
      if (grid < 1)
        return hipErrorInvalidValue;
      hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG1), lds, stream, fp, h0, gab, gcd, ge, tw, hs, HalfSlab{},
                         reinterpret_cast<unsigned char*>(spec), 1, seed);  // gcd/ge: (D, E) / C; spec: NYQ
      return hipGetLastError();
    }
  });
}

hipError_t launch_half_rows(int logn, const FrameParams& fp, const float4* gab, const float4* gcd, const float2* ge,
                            const float4* rcorr, float4* maps, float* jac, const FoamParams& foam, const float2* tw,
                            hipStream_t stream, int cus)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (!HalfCfg<LOGN>::SUPPORTED)
      return hipErrorInvalidValue;
    else
    {
      using S = FftShape<LOGN>;
      // One item = both images of its rows (C loaded once, kept in VGPRs for image 1); loads use the
      // default policy so the gc lines shared by neighbouring items survive until the partner's read
      // (streamed loads: -5 %, tools/microbench/halfbench). At N = 4096 one row per 256-thread
      // workgroup, four per CU, the 4 rows of a gc line grouped on one XCD: 1.407 -> 1.377 ms per
      // 8 x 4096^2 against two-row workgroups (halfbench rowv 16), which stay below 4096.
      constexpr int RG = kHalfRG, RGC = kHalfRGC;
      const HalfFieldLayout lay = half_rows_layout(LOGN, fp.cascades, half_rows_variant);
      if (lay.fb == 2 ? (lay.rg != kHalfRG2 || lay.rgc != kHalfRGC2) : (lay.rg != RG || lay.rgc != RGC))
        return hipErrorInvalidValue;  // the kernels below are instantiated for these two layouts only
      if constexpr (LOGN == 12)
      {
        if (half_rows_variant == 1)
        {
          // whole strips: three workgroups per CU with image 1's (D, E) loads issued before image 0's
          // stores (EARLY 1, MINB 3): 1.362 / 1.366 -> 1.345 / 1.351 ms per 8 x 4096^2 on two boxes, maps
          // bit-identical (halfbench hpe, profiles/r05_halfbench_hpe2_8.log, r05_halfbench_hpe3_8.log)
          auto kern = lay.fb == 2 ? k_rows_hp<kHalfRG2, kHalfRGC2, false, false, 2, kHalfRGC2>
                                                             : k_rows_hp<RG, RGC, false, false, 4, 4, 1, 3>;
          const int grid = persistent_grid(kern, 256, HpCfg::LDS, fp.cascades * S::N, cus);
          hipLaunchKernelGGL(kern, dim3(grid), dim3(256), HpCfg::LDS, stream, fp, gab, gcd, ge, rcorr, maps, jac, foam, tw, 0,
                             RowSrc{});
          return hipGetLastError();
        }
      }
      constexpr int RPW = LOGN == 12 ? 1 : 2, GRP = LOGN == 12 ? 4 : 2;
      // the column pass chose the field layout by cascade count (half_fields_fb): the fallback reads
      // the same one (FB = 2 with row groups 4 / 8 at 2048 / 4096 and <= 2 cascades)
      auto kern = k_rows_half<LOGN, 0, kStream, 0, RPW, true, false, RG, RGC, 4, GRP>;
      if constexpr (LOGN == 12 || LOGN == 11)
        if (lay.fb == 2)
          kern = k_rows_half<LOGN, 0, kStream, 0, RPW, true, false, kHalfRG2, kHalfRGC2, 2, GRP>;
      const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + lds_row_slots<LOGN>(RPW) * 8;
      const int grid = persistent_grid(kern, S::T * RPW, lds, fp.cascades * (S::N / RPW), cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(S::T * RPW), lds, stream, fp, gab, gcd, ge, rcorr, maps, jac, foam, tw,
                         S::N, RowSrc{}, (const float2*)nullptr);
      return hipGetLastError();
    }
  });
}

}  // namespace oceanfft

// The pairing table (include/oceanfft.h ocean_frame_plan): host only, no device needed.
extern "C" int ocean_frame_plan(size_t texture_size, int cascades, int rows_variant, int32_t out[8])
{
  using namespace oceanfft;
  int logn = 0;
  while (logn < 15 && ((size_t)1 << logn) < texture_size)
    logn++;
  if (!out || ((size_t)1 << logn) != texture_size || !half_spectrum_supported(logn) || cascades < 1 ||
      cascades > kMaxCascades || rows_variant < 0 || rows_variant > 1)
    return OCEAN_ERR_INVALID;
  const HalfFieldLayout c = half_cols_layout(logn, cascades), r = half_rows_layout(logn, cascades, rows_variant);
  const int v[8] = {c.fb, c.rg, c.rgc, c.h0_blk, r.fb, r.rg, r.rgc, half_h0_block(logn, cascades)};
  for (int k = 0; k < 8; k++)
    out[k] = v[k];
  return OCEAN_OK;
}
