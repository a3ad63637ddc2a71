// launch_common.h — host-side launch helpers shared by the kernel translation units: dispatch on
// log2 N, and grid sizing (one-shot grids on the whole device, persistent grids under a CU budget).
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>
#include <type_traits>
#include <vector>

namespace oceanfft
{

// LDS bytes of the twiddle table of an N = 2^LOGN transform, rounded to 16 B (the exchange follows it)
template <int TW_ENTRIES>
constexpr int tw_bytes() { return ((TW_ENTRIES * 8 + 15) / 16) * 16; }

template <typename F>
inline hipError_t with_logn(int logn, F&& f)
{
  switch (logn)
  {
  case 4: return f(std::integral_constant<int, 4>{});
  case 5: return f(std::integral_constant<int, 5>{});
  case 6: return f(std::integral_constant<int, 6>{});
  case 7: return f(std::integral_constant<int, 7>{});
  case 8: return f(std::integral_constant<int, 8>{});
  case 9: return f(std::integral_constant<int, 9>{});
  case 10: return f(std::integral_constant<int, 10>{});
  case 11: return f(std::integral_constant<int, 11>{});
  case 12: return f(std::integral_constant<int, 12>{});
  case 13: return f(std::integral_constant<int, 13>{});
  case 14: return f(std::integral_constant<int, 14>{});
  default: return hipErrorInvalidValue;
  }
}

// Grid sizing. With the whole device available (cus >= the device's CUs) every kernel with an item
// loop gets a one-shot grid, one block per work item: the hardware dispatcher then hands items out
// in order, so the blocks in flight at any time work on neighbouring items (adjacent strips share
// 128-B lines in L2, rows stream through neighbouring DRAM pages). Measured against persistent grids
// (resident blocks x CUs, same kernels; tools/microbench/gridbench, profiles/r02_gridbench.log):
// row pass 1.513 -> 1.453 ms, EncodeIFFT strided pass 1.115 -> 0.927 ms, 16384 column pass 6.69 ->
// 5.56 ms. Under a CU budget (ocean_fft_set_cu_budget: CUs left free for RCCL's copy kernels in
// the slab pipeline) grids stay persistent, so at most `cus` CUs' worth of blocks exist. Kernels
// with per-block scratch (the H scratch of the half-spectrum column pass) cap the grid themselves.
// The occupancy query and the dynamic-LDS attribute are set once per kernel instantiation (host API
// calls cost microseconds; a frame is two launches).
inline int device_cu_count()
{
  static const int n = [] {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return c;
  }();
  return n;
}

inline bool g_force_persistent = false;  // tools/microbench A/B only

// 4096 row pass (whole grids, launch_half_rows, and the strip-dealt slabs' row-major fields,
// launch_rm_rows): 1 = k_rows_hp (production: T_in with the mirror, 256-point sub-transforms in the
// wave through permlane / DPP swaps, T_out; device/k_rows_hp.h), 0 = k_rows_half (the mirror
// exchange, then fft_run<12>). 8 x 4096^2: 1.377 -> 1.360 ms, maps within 1e-6 of max
// (profiles/r04_halfbench_hp.log). Both paths switch together, so slabs stay bit-identical to whole grids.
inline int half_rows_variant = 1;

// Whole-grid half-spectrum fields at N = 4096 with <= 2 cascades per launch (the 4- and 8-GPU shares of
// the headline): pass 1 on half strips, two 512-thread workgroups per CU, into field strips FB = 2
// columns wide (whole-line stores: gab / gde row groups of 4, gc of 8), the row pass on that layout.
// Same per-column arithmetic as the 4-column strips, so the maps are bit-identical to them; at one
// cascade the frame takes 0.319 against 0.339 ms, at two 0.597 against 0.609, at three and more it
// loses (profiles/r04_halfbench_fb2h_{1,2,3,4,8}.log). Both launchers take the layout from here.
// N = 2048 (round 6) likewise: 256-thread half-strip workgroups, up to four per CU. At one cascade the
// 4-column pass has 257 items for 256 CUs, and the CU that runs two sets the pass's time (0.0577 ms
// against 0.0345 with 256 items, profiles/r06_halfbench_tail_11.log); the 513 half-strip items fit the
// 1024 slots at once: column pass 0.0431 -> 0.0311 ms, frame 0.0945 -> 0.0862 ms, at two cascades
// 0.1642 -> 0.1621 ms, at four it loses (0.2960 -> 0.3322), maps bit-identical
// (profiles/r06_halfbench_h2k_{1,2,4}.log).
inline int half_fields_fb(int logn, int cascades) { return (logn == 12 || logn == 11) && cascades <= 2 ? 2 : 4; }
constexpr int kHalfRG2 = 4, kHalfRGC2 = 8;  // the FB = 2 layout's row groups

// The whole-grid half-spectrum fields as one launcher writes / the other reads them: field strip width
// FB, row groups of gab / gde (RG) and of gc (RGC), and the h0 strip width. launch_half_columns and
// launch_half_rows each choose their kernel FROM their own descriptor (half_cols_layout /
// half_rows_layout, launch_half.hip), and ocean_frame_plan reports both, so a CPU test can check every
// (N, cascades, row-pass variant) pairs the layout the column pass writes with the one the row pass reads
// (the round-4 fallback row pass read the FB = 4 layout the column pass no longer wrote at <= 2 cascades).
struct HalfFieldLayout
{
  int fb, rg, rgc, h0_blk;
};


inline bool one_shot_grids(int cus)
{
  const int d = device_cu_count();
  return !g_force_persistent && d > 0 && cus >= d;
}

struct LaunchCacheEntry
{
  const void* kernel;
  int lds;
  int per_cu;
};

template <typename K>
int blocks_per_cu(K kernel, int wg, int lds)
{
  static std::mutex mu;
  static std::vector<LaunchCacheEntry> cache;
  int per_cu = -1;
  {
    std::lock_guard<std::mutex> lock(mu);
    for (const auto& e : cache)
      if (e.kernel == (const void*)kernel && e.lds == lds)
        per_cu = e.per_cu;
    if (per_cu < 0)
    {
      per_cu = 0;
      (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, wg, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
      cache.push_back({(const void*)kernel, lds, per_cu});
    }
  }
  return per_cu;
}

// Resident workgroups for `cus` CUs (at most `items`): the grid of a kernel that software-pipelines
// across the items of one workgroup (k_rows_xs EARLY 3 issues the next row's loads before the current
// row's stores), whatever one_shot_grids says.
template <typename K>
int resident_grid(K kernel, int wg, int lds, int items, int cus)
{
  long g = (long)blocks_per_cu(kernel, wg, lds) * cus;
  if (g > items)
    g = items;
  return g < 1 ? 1 : (int)g;
}

template <typename K>
int persistent_grid(K kernel, int wg, int lds, int items, int cus)
{
  if (one_shot_grids(cus))
  {
    (void)blocks_per_cu(kernel, wg, lds);  // sets the LDS attribute once
    return items < 1 ? 1 : items;
  }
  return resident_grid(kernel, wg, lds, items, cus);
}

}  // namespace oceanfft
