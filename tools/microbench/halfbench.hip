// halfbench.hip — interleaved A/B timing of half-spectrum frame-pass variants (8 cascades x 4096^2),
// with a bit-identity check of every variant's output against the baseline variant.
// Build: see Makefile target `microbench`. Usage: halfbench [logn] [cascades] [quick|mall|rows|overlap|rowabl|hpair|hp|hx|xgrid|fb2h]
#include "all_kernels.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace oceanfft;

#define CHECK(x)                                                                                   \
  do                                                                                               \
  {                                                                                                \
    hipError_t e = (x);                                                                            \
    if (e != hipSuccess)                                                                           \
    {                                                                                              \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);            \
      std::exit(1);                                                                                \
    }                                                                                              \
  } while (0)

template <typename F>
static float time_ms(F&& launch, int reps)
{
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; r++)
    CHECK(launch());
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms / reps;
}

static std::vector<unsigned char> snap(const void* d, size_t bytes)
{
  std::vector<unsigned char> h(bytes);
  CHECK(hipMemcpy(h.data(), d, bytes, hipMemcpyDeviceToHost));
  return h;
}

int main(int argc, char** argv)
{
  const int logn = argc > 1 ? std::atoi(argv[1]) : 12;
  const int C = argc > 2 ? std::atoi(argv[2]) : 8;
  const int n = 1 << logn;
  if (!half_spectrum_supported(logn))
  {
    std::printf("half path: N = 1024 .. 4096 only\n");
    return 1;
  }
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t tex = (size_t)n * n;
  float4 *h0, *maps, *gab, *gcd, *spec;
  float2 *ge, *tw, *hs;
  float* jac;
  const size_t ht = half_field_texels(logn) * C;
  CHECK(hipMalloc(&h0, tex * C * sizeof(float4)));
  CHECK(hipMalloc(&maps, tex * C * 2 * sizeof(float4)));
  CHECK(hipMalloc(&jac, tex * C * sizeof(float)));
  CHECK(hipMalloc(&gab, ht * sizeof(float4)));
  CHECK(hipMalloc(&gcd, ht * sizeof(float4)));
  CHECK(hipMalloc(&ge, ht * sizeof(float2)));
  CHECK(hipMalloc(&spec, (size_t)C * 2 * n * sizeof(float4)));
  CHECK(hipMalloc(&hs, half_hs_bytes(logn, cus)));
  int lb = logn / 2, tb = 1 << lb, ta = 1 << (logn - lb);
  std::vector<float2> tab(tb + ta);
  for (int e = 0; e < tb; e++)
    tab[e] = make_float2((float)std::cos(2 * M_PI * e / n), (float)std::sin(2 * M_PI * e / n));
  for (int e = 0; e < ta; e++)
    tab[tb + e] = make_float2((float)std::cos(2 * M_PI * e * tb / n), (float)std::sin(2 * M_PI * e * tb / n));
  CHECK(hipMalloc(&tw, tab.size() * sizeof(float2)));
  CHECK(hipMemcpy(tw, tab.data(), tab.size() * sizeof(float2), hipMemcpyHostToDevice));

  static const float planes[] = {5, 17, 101, 251, 509, 1021, 2039, 4093};
  FrameParams fp{};
  FoamParams foam{};
  fp.cascades = C;
  for (int c = 0; c < C; c++)
  {
    OceanSettings s{};
    s.seed[0] = 12342;
    s.seed[1] = 8934;
    s.U_10 = 40;
    s.theta_0 = 25;
    s.F = 800000;
    s.g = 9.8f;
    s.swell = 0.5f;
    s.h = 100;
    s.displacement = 0.4f;
    s.planeSize = planes[c % 8];
    s.scale = 1;
    s.spread = 0.2f;
    CHECK(launch_generate_spectrum(s, n, h0 + tex * c, 0, cus));
    fp.c[c] = {2.0f * 3.14159265358f / s.planeSize, 37.5f, s.g, s.h};
    foam.displacement[c] = s.displacement;
  }
  CHECK(hipDeviceSynchronize());
  const double pts = (double)tex * C;

  auto c0 = [&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus); };
  auto c1 = [&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus); };
  auto r0 = [&] { return launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus, 6); };
  auto r1 = [&] { return launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus); };
  auto r2 = [&] { return launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus, 7); };

  // bit identity: baseline frame, then each variant on the same inputs (float compare, NaN-aware)
  const size_t mb = tex * C * 2 * sizeof(float4), jb = tex * C * sizeof(float);
  auto diff = [](const std::vector<unsigned char>& a, const std::vector<unsigned char>& b) {
    const float* x = reinterpret_cast<const float*>(a.data());
    const float* y = reinterpret_cast<const float*>(b.data());
    size_t bad = 0, first = (size_t)-1;
    double worst = 0;
    for (size_t k = 0; k < a.size() / 4; k++)
      if (std::memcmp(x + k, y + k, 4) != 0)
      {
        if (first == (size_t)-1)
          first = k;
        bad++;
        worst = std::max(worst, (double)std::fabs(x[k] - y[k]));
      }
    if (bad)
      std::printf("    %zu of %zu floats differ (first at %zu: %g vs %g), max |diff| %g\n", bad, a.size() / 4, first,
                  x[first], y[first], worst);
    return bad == 0;
  };
  CHECK(c0());
  CHECK(hipDeviceSynchronize());
  auto ref_ab = snap(gab, ht * sizeof(float4)), ref_de = snap(gcd, ht * sizeof(float4)), ref_c = snap(ge, ht * sizeof(float2));
  CHECK(r0());
  CHECK(hipDeviceSynchronize());
  auto ref_m = snap(maps, mb), ref_j = snap(jac, jb);
  CHECK(hipMemset(maps, 0, mb));
  CHECK(hipMemset(jac, 0, jb));
  CHECK(r1());
  CHECK(hipDeviceSynchronize());
  std::printf("rows (both images) vs baseline on the same fields:\n");
  const bool same_rows = (int)diff(snap(maps, mb), ref_m) & (int)diff(snap(jac, jb), ref_j);
  CHECK(c0());
  CHECK(hipDeviceSynchronize());
  std::printf("cols baseline run twice:\n");
  const bool det = (int)diff(snap(gab, ht * sizeof(float4)), ref_ab) & (int)diff(snap(gcd, ht * sizeof(float4)), ref_de) &
                   (int)diff(snap(ge, ht * sizeof(float2)), ref_c);
  CHECK(hipMemset(gab, 0, ht * sizeof(float4)));
  CHECK(hipMemset(gcd, 0, ht * sizeof(float4)));
  CHECK(hipMemset(ge, 0, ht * sizeof(float2)));
  CHECK(c1());
  CHECK(hipDeviceSynchronize());
  std::printf("cols (HS) vs baseline: gab, gde, gc\n");
  const bool same_cols = (int)diff(snap(gab, ht * sizeof(float4)), ref_ab) & (int)diff(snap(gcd, ht * sizeof(float4)), ref_de) &
                         (int)diff(snap(ge, ht * sizeof(float2)), ref_c);
  std::printf("N=%d cascades=%d CUs=%d  bit-identical: cols deterministic=%s cols(HS)=%s rows(both images)=%s\n", n, C,
              cus, det ? "yes" : "NO", same_cols ? "yes" : "NO", same_rows ? "yes" : "NO");

  const bool quick = argc > 3 && std::strcmp(argv[3], "quick") == 0;  // only the blocks below
  const bool mall = argc > 3 && std::strcmp(argv[3], "mall") == 0;
  if (argc > 3 && std::strcmp(argv[3], "rows") == 0)
  {
    // row pass: interleaved row regions after the first exchange (production) against the row
    // layout (launch_half_rows ablation 15); same arithmetic, so bit-identical maps
    CHECK(c1());
    CHECK(r1());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb), pj = snap(jac, jb);
    CHECK(hipMemset(maps, 0, mb));
    auto r15 = [&] { return launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus, 15); };
    CHECK(r15());
    CHECK(hipDeviceSynchronize());
    std::printf("row layout vs interleaved rows:\n");
    const bool same = (int)diff(snap(maps, mb), pm) & (int)diff(snap(jac, jb), pj);
    std::vector<std::vector<float>> tr(2);
    for (int r = 0; r < 9; r++)
    {
      tr[0].push_back(time_ms(r1, 10));
      tr[1].push_back(time_ms(r15, 10));
    }
    for (int k = 0; k < 2; k++)
      std::sort(tr[k].begin(), tr[k].end());
    std::printf("rows, interleaved regions (production)  median %7.3f ms\n", tr[0][4]);
    std::printf("rows, row layout (round 1)              median %7.3f ms  bit-identical %s\n", tr[1][4], same ? "yes" : "NO");
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "hp") == 0 && logn == 12)
  {
    // row pass: production (k_rows_half, mirror exchange + fft_run<12>) against k_rows_hp (T_in with
    // the mirror, 256-point sub-transforms in the wave through permlane / DPP swaps, T_out). Different
    // radix order, so the maps agree to rounding, not bit for bit.
    CHECK(c1());
    CHECK(r1());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb), pj = snap(jac, jb);
    CHECK(hipMemset(maps, 0, mb));
    CHECK(hipMemset(jac, 0, jb));
    auto hpk = k_rows_hp<kHalfRG, kHalfRGC>;
    CHECK(hipFuncSetAttribute((const void*)hpk, hipFuncAttributeMaxDynamicSharedMemorySize, HpCfg::LDS));
    const int hgrid = persistent_grid(hpk, 256, HpCfg::LDS, C * n, cus);
    auto rhp = [&] {
      hipLaunchKernelGGL(hpk, dim3(hgrid), dim3(256), HpCfg::LDS, 0, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0,
                         RowSrc{});
      return hipGetLastError();
    };
    CHECK(rhp());
    CHECK(hipDeviceSynchronize());
    const auto hm = snap(maps, mb), hj = snap(jac, jb);
    const float* a = reinterpret_cast<const float*>(pm.data());
    const float* b = reinterpret_cast<const float*>(hm.data());
    double dm = 0, am = 0;
    for (size_t k = 0; k < mb / 4; k++)
    {
      dm = std::max(dm, (double)std::fabs(a[k] - b[k]));
      am = std::max(am, (double)std::fabs(a[k]));
    }
    const float* ja = reinterpret_cast<const float*>(pj.data());
    const float* jb2 = reinterpret_cast<const float*>(hj.data());
    double dj = 0, aj = 0;
    for (size_t k = 0; k < jb / 4; k++)
    {
      dj = std::max(dj, (double)std::fabs(ja[k] - jb2[k]));
      aj = std::max(aj, (double)std::fabs(ja[k]));
    }
    std::printf("k_rows_hp vs k_rows_half: maps max|diff| %.3g of max %.3g (%.2g), jacobian %.3g of %.3g (grid %d)\n", dm, am,
                dm / am, dj, aj, hgrid);
    std::vector<std::vector<float>> tr(2);
    for (int r = 0; r < 9; r++)
    {
      tr[0].push_back(time_ms(r1, 10));
      tr[1].push_back(time_ms(rhp, 10));
    }
    for (int k = 0; k < 2; k++)
      std::sort(tr[k].begin(), tr[k].end());
    std::printf("rows, k_rows_half (round 3)     median %7.3f ms  %7.1f GB/s at 56 B/pt\n", tr[0][4], 56.04 * pts / tr[0][4] / 1e6);
    std::printf("rows, k_rows_hp (permlane/DPP) median %7.3f ms  %7.1f GB/s at 56 B/pt\n", tr[1][4], 56.04 * pts / tr[1][4] / 1e6);
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "hx") == 0 && logn == 12)
  {
    // pass 1: production (fft_run<12>: two split LDS exchanges, 8 barriers per round) against HX (one
    // LDS exchange + the in-wave transposition of lane_xchg.h, 4 barriers). HX 1 stores rows w + 16 a +
    // 256 m (half lines per store instruction), HX 2 stores them in storage-row order (whole lines;
    // the row pass k_rows_hp YP reads storage rows). Different radix order, so the maps agree to
    // rounding, not bit for bit. Frames with k_rows_hp.
    using K = ColFirstCfg<12>;
    using S = FftShape<12>;
    const int clds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + K::LDS1 + kHalfHL * K::WG1 * 16;
    auto cols = [&](auto kern) {
      return std::function<hipError_t()>([=] {
        hipError_t e = launch_half_nyquist(fp, n, K::B, h0, spec, nullptr, 1, 0, nullptr, 0, cus);
        if (e != hipSuccess)
          return e;
        int grid = persistent_grid(kern, K::WG1, clds, fp.cascades * HalfCfg<12>::STRIPS, cus);
        grid = grid > cus ? cus : grid;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG1), clds, 0, fp, h0, gab, gcd, ge, tw, hs, HalfSlab{},
                           (unsigned char*)nullptr, 1, nullptr);
        return hipGetLastError();
      });
    };
    auto rows = [&](auto kern) {
      return std::function<hipError_t()>([=] {
        const int grid = persistent_grid(kern, 256, HpCfg::LDS, fp.cascades * n, cus);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), HpCfg::LDS, 0, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0,
                           RowSrc{});
        return hipGetLastError();
      });
    };
    auto rp = rows(k_rows_hp<kHalfRG, kHalfRGC>), ry = rows(k_rows_hp<kHalfRG, kHalfRGC, false, true>);
    std::vector<std::function<hipError_t()>> vc = {
        cols(k_cols_half<12, kStream, kStream, true, false, false, kHalfRG, kHalfRGC, 4, true, false, kHalfHL, kHalfHK>),
        cols(k_cols_half<12, kStream, kStream, true, false, false, kHalfRG, kHalfRGC, 4, true, false, kHalfHL, kHalfHK, 1>),
        cols(k_cols_half<12, kStream, kStream, true, false, false, kHalfRG, kHalfRGC, 4, true, false, kHalfHL, kHalfHK, 2>),
        cols(k_cols_half<12, kStream, kStream, true, false, false, kHalfRG, kHalfRGC, 4, true, false, kHalfHL, 2, 2>)};
    std::vector<std::function<hipError_t()>> vr = {rp, rp, ry, ry};
    const char* nm[] = {"production (fft_run, HK 4)", "HX 1 (row order), HK 4", "HX 2 (storage order), HK 4",
                        "HX 2 (storage order), HK 2"};
    const int NV = 4;
    auto rel = [](const std::vector<unsigned char>& a, const std::vector<unsigned char>& b) {
      const float* x = reinterpret_cast<const float*>(a.data());
      const float* y = reinterpret_cast<const float*>(b.data());
      double d = 0, m = 0;
      for (size_t k = 0; k < a.size() / 4; k++)
      {
        d = std::max(d, (double)std::fabs(x[k] - y[k]));
        m = std::max(m, (double)std::fabs(x[k]));
      }
      return d / (m > 0 ? m : 1);
    };
    CHECK(vc[0]());
    CHECK(vr[0]());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb), pj = snap(jac, jb);
    for (int k = 1; k < NV; k++)
    {
      CHECK(hipMemset(maps, 0, mb));
      CHECK(hipMemset(jac, 0, jb));
      CHECK(vc[k]());
      CHECK(vr[k]());
      CHECK(hipDeviceSynchronize());
      std::printf("%s vs production: maps %.2g jacobian %.2g (max |diff| / max)\n", nm[k], rel(snap(maps, mb), pm),
                  rel(snap(jac, jb), pj));
    }
    std::vector<std::vector<float>> t(NV), tr(NV), tf(NV);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < NV; k++)
      {
        t[k].push_back(time_ms(vc[k], 10));
        tr[k].push_back(time_ms(vr[k], 10));
        tf[k].push_back(time_ms([&] { CHECK(vc[k]()); return vr[k](); }, 10));
      }
    for (int k = 0; k < NV; k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::sort(tr[k].begin(), tr[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("cols %-28s median %7.3f ms  %7.1f GB/s at 28 B/pt   rows %7.3f ms   frame %7.3f ms\n", nm[k], t[k][4],
                  28.0 * pts / t[k][4] / 1e6, tr[k][4], tf[k][4]);
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "rg") == 0 && logn == 12)
  {
    // the gab / gde row-group size RG (gc keeps RGC = 4) with the production row pass (one row per
    // 256-thread workgroup, 4 rows per XCD group, so a 128-B line's two rows stay on one XCD for any
    // RG >= 2): pass 1's store pieces are RG x 64 B. Same arithmetic, so the maps must be identical.
    using K = ColFirstCfg<12>;
    using S = FftShape<12>;
    const int clds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + K::LDS1 + kHalfHL * K::WG1 * 16;
    const int rlds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + lds_row_slots<12>(1) * 8;
    auto cols = [&](auto kern) {
      return [=] {
        hipError_t e = launch_half_nyquist(fp, n, K::B, h0, spec, nullptr, 1, 0, nullptr, 0, cus);
        if (e != hipSuccess)
          return e;
        int grid = persistent_grid(kern, K::WG1, clds, fp.cascades * HalfCfg<12>::STRIPS, cus);
        grid = grid > cus ? cus : grid;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG1), clds, 0, fp, h0, gab, gcd, ge, tw, hs, HalfSlab{},
                           (unsigned char*)nullptr, 1, nullptr);
        return hipGetLastError();
      };
    };
    auto rows = [&](auto kern) {
      return [=] {
        const int grid = persistent_grid(kern, S::T, rlds, fp.cascades * S::N, cus);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(S::T), rlds, 0, fp, gab, gcd, ge, spec, maps, jac, foam, tw, S::N,
                           RowSrc{}, (const float2*)nullptr);
        return hipGetLastError();
      };
    };
    std::vector<std::function<hipError_t()>> vc = {
        cols(k_cols_half<12, kStream, kStream, true, false, false, 2, 4, 4, true, false, kHalfHL, kHalfHK>),
        cols(k_cols_half<12, kStream, kStream, true, false, false, 4, 4, 4, true, false, kHalfHL, kHalfHK>),
        cols(k_cols_half<12, kStream, kStream, true, false, false, 8, 4, 4, true, false, kHalfHL, kHalfHK>),
        cols(k_cols_half<12, kStream, kStream, true, false, false, 16, 4, 4, true, false, kHalfHL, kHalfHK>)};
    std::vector<std::function<hipError_t()>> vr = {
        rows(k_rows_half<12, 0, kStream, 0, 1, true, false, 2, 4, 4, 4>),
        rows(k_rows_half<12, 0, kStream, 0, 1, true, false, 4, 4, 4, 4>),
        rows(k_rows_half<12, 0, kStream, 0, 1, true, false, 8, 4, 4, 4>),
        rows(k_rows_half<12, 0, kStream, 0, 1, true, false, 16, 4, 4, 4>)};
    const int rgs[4] = {2, 4, 8, 16};
    CHECK(vc[0]());
    CHECK(vr[0]());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb), pj = snap(jac, jb);
    bool same[4] = {true, true, true, true};
    for (int k = 1; k < 4; k++)
    {
      CHECK(hipMemset(maps, 0, mb));
      CHECK(vc[k]());
      CHECK(vr[k]());
      CHECK(hipDeviceSynchronize());
      std::printf("RG %d vs RG 2: maps, jacobian\n", rgs[k]);
      same[k] = (int)diff(snap(maps, mb), pm) & (int)diff(snap(jac, jb), pj);
    }
    std::vector<std::vector<float>> tc(4), tr(4), tf(4);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < 4; k++)
      {
        tc[k].push_back(time_ms(vc[k], 10));
        tr[k].push_back(time_ms(vr[k], 10));
        auto fr = [&] { CHECK(vc[k]()); return vr[k](); };
        tf[k].push_back(time_ms(fr, 10));
      }
    for (int k = 0; k < 4; k++)
    {
      std::sort(tc[k].begin(), tc[k].end());
      std::sort(tr[k].begin(), tr[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("RG %2d (gab/gde pieces %4d B)  cols %7.3f  rows %7.3f  frame %7.3f ms  bit-identical %s%s\n", rgs[k],
                  rgs[k] * 64, tc[k][4], tr[k][4], tf[k][4], same[k] ? "yes" : "NO", k == 0 ? " (production)" : "");
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "hpair") == 0)
  {
    // pass 1 with the H scratch in 8-B entries (variant 23, round 2) against production (16-B pairs):
    // bit-identical fields
    auto cp = [&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus, nullptr, 23); };
    CHECK(c1());
    CHECK(hipDeviceSynchronize());
    auto pab = snap(gab, ht * sizeof(float4)), pde = snap(gcd, ht * sizeof(float4)), pc = snap(ge, ht * sizeof(float2));
    CHECK(hipMemset(gab, 0, ht * sizeof(float4)));
    CHECK(hipMemset(gcd, 0, ht * sizeof(float4)));
    CHECK(hipMemset(ge, 0, ht * sizeof(float2)));
    CHECK(cp());
    CHECK(hipDeviceSynchronize());
    std::printf("cols with unpaired H scratch vs production: gab, gde, gc\n");
    const bool same = (int)diff(snap(gab, ht * sizeof(float4)), pab) & (int)diff(snap(gcd, ht * sizeof(float4)), pde) &
                      (int)diff(snap(ge, ht * sizeof(float2)), pc);
    std::vector<std::vector<float>> t(2);
    for (int r = 0; r < 9; r++)
    {
      t[0].push_back(time_ms(c1, 10));
      t[1].push_back(time_ms(cp, 10));
    }
    for (auto& v : t)
      std::sort(v.begin(), v.end());
    std::printf("cols (production, pairs)   median %7.3f ms\n", t[0][4]);
    std::printf("cols, unpaired H scratch   median %7.3f ms  bit-identical %s\n", t[1][4], same ? "yes" : "NO");
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "packc") == 0)
  {
    // pass 1 with round 2's (C, 0) CPairs packed as column pairs on half the workgroup (variant 24)
    // against production: bit-identical fields (same per-lane arithmetic)
    auto cp = [&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus, nullptr, 24); };
    CHECK(c1());
    CHECK(hipDeviceSynchronize());
    auto pab = snap(gab, ht * sizeof(float4)), pde = snap(gcd, ht * sizeof(float4)), pc = snap(ge, ht * sizeof(float2));
    CHECK(hipMemset(gab, 0, ht * sizeof(float4)));
    CHECK(hipMemset(gcd, 0, ht * sizeof(float4)));
    CHECK(hipMemset(ge, 0, ht * sizeof(float2)));
    CHECK(cp());
    CHECK(hipDeviceSynchronize());
    std::printf("cols with the packed C round vs production: gab, gde, gc\n");
    const bool same = (int)diff(snap(gab, ht * sizeof(float4)), pab) & (int)diff(snap(gcd, ht * sizeof(float4)), pde) &
                      (int)diff(snap(ge, ht * sizeof(float2)), pc);
    std::vector<std::vector<float>> t(4);
    for (int r = 0; r < 9; r++)
    {
      t[0].push_back(time_ms(c1, 10));
      t[1].push_back(time_ms(cp, 10));
      t[2].push_back(time_ms([&] { CHECK(c1()); return r1(); }, 10));
      t[3].push_back(time_ms([&] { CHECK(cp()); return r1(); }, 10));
    }
    for (auto& v : t)
      std::sort(v.begin(), v.end());
    std::printf("cols (production)          median %7.3f ms   frame %7.3f ms\n", t[0][4], t[2][4]);
    std::printf("cols, packed C round       median %7.3f ms   frame %7.3f ms  bit-identical %s\n", t[1][4], t[3][4],
                same ? "yes" : "NO");
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "cap") == 0)
  {
    // pass 1 below 4096: grid capped at one H-scratch slice per 1024 threads (production: 1024 / WG1
    // blocks per slice, so 2048 runs two workgroups per CU and 1024 four) against one block per slice
    // (variant 37, round 2's earlier cap); same kernel, same fields
    auto cp = [&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus, nullptr, 37); };
    CHECK(c1());
    CHECK(hipDeviceSynchronize());
    auto pab = snap(gab, ht * sizeof(float4)), pde = snap(gcd, ht * sizeof(float4)), pc = snap(ge, ht * sizeof(float2));
    CHECK(hipMemset(gab, 0, ht * sizeof(float4)));
    CHECK(hipMemset(gcd, 0, ht * sizeof(float4)));
    CHECK(hipMemset(ge, 0, ht * sizeof(float2)));
    CHECK(cp());
    CHECK(hipDeviceSynchronize());
    std::printf("cols, one block per scratch slice vs production: gab, gde, gc\n");
    const bool same = (int)diff(snap(gab, ht * sizeof(float4)), pab) & (int)diff(snap(gcd, ht * sizeof(float4)), pde) &
                      (int)diff(snap(ge, ht * sizeof(float2)), pc);
    std::vector<std::vector<float>> t(4);
    for (int r = 0; r < 9; r++)
    {
      t[0].push_back(time_ms(c1, 10));
      t[1].push_back(time_ms(cp, 10));
      t[2].push_back(time_ms([&] { CHECK(c1()); return r1(); }, 10));
      t[3].push_back(time_ms([&] { CHECK(cp()); return r1(); }, 10));
    }
    for (auto& v : t)
      std::sort(v.begin(), v.end());
    std::printf("N=%d x %d  cols (production)            median %7.3f ms   frame %7.3f ms\n", n, C, t[0][4], t[2][4]);
    std::printf("N=%d x %d  cols, one block per slice    median %7.3f ms   frame %7.3f ms  bit-identical %s\n", n, C,
                t[1][4], t[3][4], same ? "yes" : "NO");
    return 0;
  }
  if (argc > 4 && std::strcmp(argv[3], "rowv") == 0)
  {
    // row-pass variants (launch_half_rows ablation numbers from the command line) against production
    // on the same fields: timing, and maps/Jacobian bit-identity
    CHECK(c1());
    CHECK(r1());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb), pj = snap(jac, jb);
    std::vector<int> av{0};
    for (int a = 4; a < argc; a++)
      av.push_back(std::atoi(argv[a]));
    std::vector<int> same(av.size(), 1);
    for (size_t k = 1; k < av.size(); k++)
    {
      CHECK(hipMemset(maps, 0, mb));
      CHECK(hipMemset(jac, 0, jb));
      CHECK(launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus, av[k]));
      CHECK(hipDeviceSynchronize());
      std::printf("rows variant %d vs production: maps, jacobian\n", av[k]);
      same[k] = (int)diff(snap(maps, mb), pm) & (int)diff(snap(jac, jb), pj);
    }
    std::vector<std::vector<float>> t(av.size());
    for (int r = 0; r < 9; r++)
      for (size_t k = 0; k < av.size(); k++)
        t[k].push_back(time_ms([&] { return launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus, av[k]); }, 10));
    for (size_t k = 0; k < av.size(); k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::printf("rows variant %2d  median %7.3f ms  %7.1f GB/s at 56 B/pt  bit-identical %s\n", av[k], t[k][4],
                  56.04 * pts / t[k][4] / 1e6, same[k] ? "yes" : "NO");
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "fb2") == 0)
  {
    // half-strip pass 1 (k_cols_half2: 2 columns per 512-thread item, H in VGPRs, no H scratch) with
    // the one-row pass 2 on the FB = 2 layouts (rows variants 18 / 19), against production
    const int BIG = 1 << 20;
    CHECK(c1());
    CHECK(r1());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb), pj = snap(jac, jb);
    struct V
    {
      const char* name;
      int cv, rv, cus;
    };
    const V vs[] = {{"production", 0, 0, 0},
                    {"half2 RG4/RGC8 persistent + rows 18", 12, 18, cus},
                    {"half2 RG4/RGC8 one-shot + rows 18", 12, 18, BIG},
                    {"half2 RG4/RGC4 persistent + rows 19", 14, 19, cus},
                    {"half2 RG4/RGC8 persistent + rows 12 (2-row)", 12, 12, cus}};
    const int NV = sizeof(vs) / sizeof(vs[0]);
    auto cl = [&](const V& v) {
      return [&, v] {
        return v.cv == 0 ? c1() : launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, v.cus, nullptr, 0, nullptr, v.cv);
      };
    };
    auto rl = [&](const V& v) {
      return [&, v] { return v.rv == 0 ? r1() : launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus, v.rv); };
    };
    for (int k = 1; k < NV; k++)
    {
      CHECK(hipMemset(maps, 0, mb));
      CHECK(hipMemset(jac, 0, jb));
      CHECK(cl(vs[k])());
      CHECK(rl(vs[k])());
      CHECK(hipDeviceSynchronize());
      auto m = snap(maps, mb), j = snap(jac, jb);
      const float* a = reinterpret_cast<const float*>(m.data());
      const float* b = reinterpret_cast<const float*>(pm.data());
      double mx = 0, dm = 0;
      for (size_t e = 0; e < mb / 4; e++)
      {
        mx = std::max(mx, (double)std::fabs(b[e]));
        dm = std::max(dm, (double)std::fabs(a[e] - b[e]));
      }
      std::printf("%s vs production: maps max|diff| %g of max %g (%.2e)\n", vs[k].name, dm, mx, dm / mx);
      diff(j, pj);
    }
    std::vector<std::vector<float>> tc(NV), tr(NV), tf(NV);
    for (int r = 0; r < 7; r++)
      for (int k = 0; k < NV; k++)
      {
        auto c = cl(vs[k]);
        auto w = rl(vs[k]);
        tc[k].push_back(time_ms(c, 10));
        tr[k].push_back(time_ms(w, 10));
        tf[k].push_back(time_ms([&] { hipError_t e = c(); return e == hipSuccess ? w() : e; }, 10));
      }
    for (int k = 0; k < NV; k++)
    {
      std::sort(tc[k].begin(), tc[k].end());
      std::sort(tr[k].begin(), tr[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("%-46s cols %7.3f  rows %7.3f  frame %7.3f ms (median)\n", vs[k].name, tc[k][3], tr[k][3], tf[k][3]);
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "layout2") == 0)
  {
    // field layouts (RG, RGC) re-measured with production's pass 1 (5 of 8 H pairs out of the
    // scratch): pass 1 variants 34..36 with pass 2 variants 8, 10, 11; same arithmetic, so the maps
    // must be bit-identical to production's
    const int cv[4] = {0, 34, 35, 36}, rv[4] = {0, 8, 10, 11};
    const char* ln[4] = {"(2, 4) production", "(2, 2)", "(4, 4)", "(1, 1) strips"};
    CHECK(c1());
    CHECK(r1());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb), pj = snap(jac, jb);
    bool same[4] = {true, true, true, true};
    for (int v = 1; v < 4; v++)
    {
      CHECK(hipMemset(maps, 0, mb));
      CHECK(launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus, nullptr, cv[v]));
      CHECK(launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus, rv[v]));
      CHECK(hipDeviceSynchronize());
      std::printf("layout %s vs production: maps, jacobian\n", ln[v]);
      same[v] = (int)diff(snap(maps, mb), pm) & (int)diff(snap(jac, jb), pj);
    }
    std::vector<std::vector<float>> tc(4), tr(4), tf(4);
    for (int r = 0; r < 9; r++)
      for (int v = 0; v < 4; v++)
      {
        auto cl = [&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus, nullptr, cv[v]); };
        auto rl = [&] { return launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus, rv[v]); };
        tc[v].push_back(time_ms(cl, 10));
        tr[v].push_back(time_ms(rl, 10));
        tf[v].push_back(time_ms([&] { CHECK(cl()); return rl(); }, 10));
      }
    for (int v = 0; v < 4; v++)
    {
      std::sort(tc[v].begin(), tc[v].end());
      std::sort(tr[v].begin(), tr[v].end());
      std::sort(tf[v].begin(), tf[v].end());
      std::printf("%-20s cols %7.3f  rows %7.3f  frame %7.3f ms (median)  bit-identical %s\n", ln[v], tc[v][4], tr[v][4],
                  tf[v][4], same[v] ? "yes" : "NO");
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "seed") == 0)
  {
    // the fused re-seed pass 1 (h0 evaluated in round 0): production (H pairs in LDS / VGPRs /
    // scratch) against variant 33 (all 8 pairs in the scratch); same evaluator, same fields
    std::vector<SpectrumConsts> sc(C);
    for (int c = 0; c < C; c++)
    {
      OceanSettings s{};
      s.seed[0] = 12342;
      s.seed[1] = 8934;
      s.U_10 = 40;
      s.theta_0 = 25;
      s.F = 800000;
      s.g = 9.8f;
      s.swell = 0.5f;
      s.h = 100;
      s.displacement = 0.4f;
      s.planeSize = planes[c % 8];
      s.scale = 1;
      s.spread = 0.2f;
      seed_consts(s, n, &sc[c]);
    }
    SpectrumConsts* dsc;
    CHECK(hipMalloc(&dsc, C * sizeof(SpectrumConsts)));
    CHECK(hipMemcpy(dsc, sc.data(), C * sizeof(SpectrumConsts), hipMemcpyHostToDevice));
    auto sv = [&](int v) { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus, dsc, v); };
    CHECK(sv(33));
    CHECK(hipDeviceSynchronize());
    auto pab = snap(gab, ht * sizeof(float4)), pde = snap(gcd, ht * sizeof(float4)), pc = snap(ge, ht * sizeof(float2));
    CHECK(hipMemset(gab, 0, ht * sizeof(float4)));
    CHECK(hipMemset(gcd, 0, ht * sizeof(float4)));
    CHECK(hipMemset(ge, 0, ht * sizeof(float2)));
    CHECK(sv(0));
    CHECK(hipDeviceSynchronize());
    std::printf("re-seed cols, production vs variant 33: gab, gde, gc\n");
    const bool same = (int)diff(snap(gab, ht * sizeof(float4)), pab) & (int)diff(snap(gcd, ht * sizeof(float4)), pde) &
                      (int)diff(snap(ge, ht * sizeof(float2)), pc);
    std::vector<std::vector<float>> t(2);
    for (int r = 0; r < 9; r++)
    {
      t[0].push_back(time_ms([&] { return sv(33); }, 10));
      t[1].push_back(time_ms([&] { return sv(0); }, 10));
    }
    for (auto& v : t)
      std::sort(v.begin(), v.end());
    std::printf("re-seed cols, 8 pairs in scratch (33)  median %7.3f ms\n", t[0][4]);
    std::printf("re-seed cols, production              median %7.3f ms  bit-identical %s\n", t[1][4], same ? "yes" : "NO");
    return 0;
  }
  if (argc > 3 && (std::strcmp(argv[3], "hs4") == 0 || std::strcmp(argv[3], "hpf") == 0) && logn == 12)
  {
    // half-strip pass 1 (two 512-thread workgroups per CU) reading 2-column h0 strips (HB 2) into the
    // whole strips' 4-column fields (FB 4: each 128-B line written as two 64-B halves by the two items
    // of a strip, on one XCD), so the production row pass reads them; against production and against
    // the FB 2 fields (whole-line stores, k_rows_hp FB 2). Maps compared with production's.
    using K = ColFirstCfg<12>;
    using S = FftShape<12>;
    float4* h0b2;
    CHECK(hipMalloc(&h0b2, tex * C * sizeof(float4)));
    for (int c = 0; c < C; c++)
    {
      OceanSettings s{};
      s.seed[0] = 12342;
      s.seed[1] = 8934;
      s.U_10 = 40;
      s.theta_0 = 25;
      s.F = 800000;
      s.g = 9.8f;
      s.swell = 0.5f;
      s.h = 100;
      s.displacement = 0.4f;
      s.planeSize = planes[c % 8];
      s.scale = 1;
      s.spread = 0.2f;
      CHECK(launch_generate_spectrum(s, n, h0b2 + tex * c, 0, cus, 0, 0, 2));
    }
    const int tw0 = ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
    const int lds4 = tw0 + K::LDS1 + kHalfHL * 1024 * 16, lds2 = tw0 + 2 * S::PADDED * 8 + kHalfHL * 512 * 16;
    auto cols = [&](auto kern, int wg, int lds, const float4* hsrc, int hb) {
      return std::function<hipError_t()>([=] {
        hipError_t e = launch_half_nyquist(fp, n, hb, hsrc, spec, nullptr, 1, 0, nullptr, 0, cus);
        if (e != hipSuccess)
          return e;
        const int items = fp.cascades * HalfCfg<12>::STRIPS * (K::WG1 / wg);
        int grid = persistent_grid(kern, wg, lds, items, cus);
        const int slices = cus * (1024 / wg);
        grid = grid > slices ? slices : grid;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(wg), lds, 0, fp, hsrc, gab, gcd, ge, tw, hs, HalfSlab{},
                           (unsigned char*)nullptr, 1, nullptr);
        return hipGetLastError();
      });
    };
    auto rows = [&](auto kern) {
      return std::function<hipError_t()>([=] {
        const int grid = persistent_grid(kern, 256, HpCfg::LDS, fp.cascades * n, cus);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), HpCfg::LDS, 0, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0,
                           RowSrc{});
        return hipGetLastError();
      });
    };
    const bool hpf = std::strcmp(argv[3], "hpf") == 0;  // the FB 2 row pass variants instead
    auto c2 = cols(k_cols_half<12, kStream, kStream, true, false, false, kHalfRG2, kHalfRGC2, 2, true, false, kHalfHL, 4, 0, 2, false, 2>, 512, lds2, h0b2, 2);
    std::vector<std::function<hipError_t()>> vc = hpf ? std::vector<std::function<hipError_t()>>{c2, c2, c2} : std::vector<std::function<hipError_t()>>{
        cols(k_cols_half<12, kStream, kStream, true, false, false, kHalfRG, kHalfRGC, 4, true, false, kHalfHL, kHalfHK>, 1024, lds4, h0, 4),
        cols(k_cols_half<12, kStream, kStream, true, false, false, kHalfRG, kHalfRGC, 2, true, false, kHalfHL, 4, 0, 4, false, 2>, 512, lds2, h0b2, 2),
        c2};
    std::vector<std::function<hipError_t()>> vr = hpf ? std::vector<std::function<hipError_t()>>{
        rows(k_rows_hp<kHalfRG2, kHalfRGC2, false, false, 2, kHalfRGC2>),
        rows(k_rows_hp<kHalfRG2, kHalfRGC2, false, false, 2, kHalfRGC2, 1, 3>),
        rows(k_rows_hp<kHalfRG2, kHalfRGC2, false, false, 2, kHalfRGC2, 0, 3>)} : std::vector<std::function<hipError_t()>>{
        rows(k_rows_hp<kHalfRG, kHalfRGC>), rows(k_rows_hp<kHalfRG, kHalfRGC>),
        rows(k_rows_hp<kHalfRG2, kHalfRGC2, false, false, 2, kHalfRGC2>)};
    const char* nm0[] = {"production (whole strips)", "half strips, h0 HB 2, fields FB 4", "half strips, h0 HB 2, fields FB 2"};
    const char* nm1[] = {"FB 2 rows (production <= 2 casc.)", "FB 2 rows, 3 WG/CU EARLY 1", "FB 2 rows, 3 WG/CU"};
    const char* const* nm = hpf ? nm1 : nm0;
    const int NV = 3;
    CHECK(vc[0]());
    CHECK(vr[0]());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb), pj = snap(jac, jb);
    for (int k = 1; k < NV; k++)
    {
      CHECK(hipMemset(maps, 0, mb));
      CHECK(hipMemset(jac, 0, jb));
      CHECK(vc[k]());
      CHECK(vr[k]());
      CHECK(hipDeviceSynchronize());
      std::printf("%s vs production: maps, jacobian\n", nm[k]);
      (void)((int)diff(snap(maps, mb), pm) & (int)diff(snap(jac, jb), pj));
    }
    std::vector<std::vector<float>> t(NV), tr(NV), tf(NV);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < NV; k++)
      {
        t[k].push_back(time_ms(vc[k], 10));
        tr[k].push_back(time_ms(vr[k], 10));
        tf[k].push_back(time_ms([&] { CHECK(vc[k]()); return vr[k](); }, 10));
      }
    for (int k = 0; k < NV; k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::sort(tr[k].begin(), tr[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("%-36s cols %7.3f ms  rows %7.3f ms  frame %7.3f ms\n", nm[k], t[k][4], tr[k][4], tf[k][4]);
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "cole") == 0 && logn == 12)
  {
    // k_cols_half with loads issued before the round's stores (EARLY bits: 1 the next round's scratch
    // pairs, 2 / 4 the next item's first 8 / 16 h0 texels) against production: fields bit-identical
    using K = ColFirstCfg<12>;
    using S = FftShape<12>;
    const int lds4 = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + K::LDS1 + kHalfHL * 1024 * 16;
    auto cols = [&](auto kern) {
      return std::function<hipError_t()>([=] {
        hipError_t e = launch_half_nyquist(fp, n, K::B, h0, spec, nullptr, 1, 0, nullptr, 0, cus);
        if (e != hipSuccess)
          return e;
        int grid = persistent_grid(kern, 1024, lds4, fp.cascades * HalfCfg<12>::STRIPS, cus);
        grid = grid > cus ? cus : grid;  // hs: cus slices of 16 x 1024 entries
        hipLaunchKernelGGL(kern, dim3(grid), dim3(1024), lds4, 0, fp, h0, gab, gcd, ge, tw, hs, HalfSlab{},
                           (unsigned char*)nullptr, 1, nullptr);
        return hipGetLastError();
      });
    };
#define KCH(E) k_cols_half<12, kStream, kStream, true, false, false, kHalfRG, kHalfRGC, 4, true, false, kHalfHL, kHalfHK, 0, 4, false, 4, E>
    std::vector<std::function<hipError_t()>> vc = {cols(KCH(0)), cols(KCH(1)), cols(KCH(2)), cols(KCH(3)), cols(KCH(4)),
                                                   cols(KCH(5))};
#undef KCH
    const char* nm[] = {"production", "EARLY 1 (scratch pairs)", "EARLY 2 (8 h0 texels)", "EARLY 3 (1 + 2)",
                        "EARLY 4 (16 h0 texels)", "EARLY 5 (1 + 4)"};
    const int NV = 6;
    CHECK(vc[0]());
    CHECK(hipDeviceSynchronize());
    auto pab = snap(gab, ht * sizeof(float4)), pde = snap(gcd, ht * sizeof(float4)), pc = snap(ge, ht * sizeof(float2));
    std::vector<int> same(NV, 1);
    for (int k = 1; k < NV; k++)
    {
      CHECK(hipMemset(gab, 0, ht * sizeof(float4)));
      CHECK(hipMemset(gcd, 0, ht * sizeof(float4)));
      CHECK(hipMemset(ge, 0, ht * sizeof(float2)));
      CHECK(vc[k]());
      CHECK(hipDeviceSynchronize());
      std::printf("%s vs production: gab, gde, gc\n", nm[k]);
      same[k] = (int)diff(snap(gab, ht * sizeof(float4)), pab) & (int)diff(snap(gcd, ht * sizeof(float4)), pde) &
                (int)diff(snap(ge, ht * sizeof(float2)), pc);
    }
    std::vector<std::vector<float>> t(NV), tf(NV);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < NV; k++)
      {
        t[k].push_back(time_ms(vc[k], 10));
        tf[k].push_back(time_ms([&] { CHECK(vc[k]()); return r1(); }, 10));
      }
    for (int k = 0; k < NV; k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("cols %-26s median %7.3f ms   frame %7.3f ms  bit-identical %s\n", nm[k], t[k][4], tf[k][4],
                  same[k] ? "yes" : "NO");
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "qx") == 0 && logn == 12)
  {
    // round 6: k_cols_half with quarter LDS exchanges (QX) so that all 8 H pairs stay on the CU (HL in
    // the LDS + HK in VGPRs, no scratch), optionally with the next item's h0 loads before round 2's
    // stores (EARLY 2 / 4), against production (HL 1 HK 4, split exchanges, 3 pairs in the scratch)
    using S = FftShape<12>;
    auto cols = [&](auto kern, int hl, bool qx) {
      const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + 4 * S::PADDED * (qx ? 4 : 8) + hl * 1024 * 16;
      return std::function<hipError_t()>([=] {
        int grid = persistent_grid(kern, 1024, lds, fp.cascades * HalfCfg<12>::STRIPS, cus);
        grid = grid > cus ? cus : grid;  // hs: cus slices of 16 x 1024 entries
        hipLaunchKernelGGL(kern, dim3(grid), dim3(1024), lds, 0, fp, h0, gab, gcd, ge, tw, hs, HalfSlab{},
                           (unsigned char*)spec, 1, nullptr);
        return hipGetLastError();
      });
    };
#define KQ(HL, HK, E, QX) k_cols_half<12, kStream, kStream, true, false, false, kHalfRG, kHalfRGC, 4, true, false, HL, HK, 0, 4, false, 4, E, true, QX>
    std::vector<std::function<hipError_t()>> vc = {cols(KQ(1, 4, 0, false), 1, false), cols(KQ(1, 4, 0, true), 1, true),
                                                   cols(KQ(4, 4, 0, true), 4, true),  cols(KQ(5, 3, 0, true), 5, true),
                                                   cols(KQ(5, 3, 2, true), 5, true),  cols(KQ(4, 4, 2, true), 4, true),
                                                   cols(KQ(5, 3, 4, true), 5, true)};
#undef KQ
    const char* nm[] = {"production (HL1 HK4)", "QX HL1 HK4", "QX HL4 HK4 (no scratch)", "QX HL5 HK3 (no scratch)",
                        "QX HL5 HK3 EARLY 2", "QX HL4 HK4 EARLY 2", "QX HL5 HK3 EARLY 4"};
    const int NV = 7;
    CHECK(vc[0]());
    CHECK(hipDeviceSynchronize());
    auto pab = snap(gab, ht * sizeof(float4)), pde = snap(gcd, ht * sizeof(float4)), pc = snap(ge, ht * sizeof(float2));
    std::vector<int> same(NV, 1);
    for (int k = 1; k < NV; k++)
    {
      CHECK(hipMemset(gab, 0, ht * sizeof(float4)));
      CHECK(hipMemset(gcd, 0, ht * sizeof(float4)));
      CHECK(hipMemset(ge, 0, ht * sizeof(float2)));
      CHECK(vc[k]());
      CHECK(hipDeviceSynchronize());
      std::printf("%s vs production: gab, gde, gc\n", nm[k]);
      same[k] = (int)diff(snap(gab, ht * sizeof(float4)), pab) & (int)diff(snap(gcd, ht * sizeof(float4)), pde) &
                (int)diff(snap(ge, ht * sizeof(float2)), pc);
    }
    std::vector<std::vector<float>> t(NV), tf(NV);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < NV; k++)
      {
        t[k].push_back(time_ms(vc[k], 10));
        tf[k].push_back(time_ms([&] { CHECK(vc[k]()); return r1(); }, 10));
      }
    for (int k = 0; k < NV; k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("cols %-28s median %7.3f ms (%6.1f GB/s at 28.05 B/pt)  frame %7.3f ms  bit-identical %s\n", nm[k],
                  t[k][4], 28.05 * pts / t[k][4] / 1e6, tf[k][4], same[k] ? "yes" : "NO");
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "h2k") == 0 && logn == 11)
  {
    // round 6: N = 2048 on half strips (2-column items of 256 threads, up to four per CU, FB = 2 fields,
    // 2-column h0 strips) against production (4-column items of 512 threads, two per CU): at one cascade
    // the production pass has 257 items for 256 CUs, so one CU runs two and the pass takes ~1.7 items'
    // time (halfbench tail); the half-strip pass spreads 513 items over 1024 slots. Maps compared.
    using S = FftShape<11>;
    float4* h02;
    CHECK(hipMalloc(&h02, tex * C * sizeof(float4)));
    for (int c = 0; c < C; c++)
    {
      OceanSettings st{};
      st.seed[0] = 12342; st.seed[1] = 8934; st.U_10 = 40; st.theta_0 = 25; st.F = 800000; st.g = 9.8f;
      st.swell = 0.5f; st.h = 100; st.displacement = 0.4f; st.planeSize = planes[c % 8]; st.scale = 1; st.spread = 0.2f;
      CHECK(launch_generate_spectrum(st, n, h02 + tex * c, 0, cus, 0, 0, 2));
    }
    auto prod_c = [&] { return launch_half_columns(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus); };
    auto prod_r = [&] { return launch_half_rows(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus); };
    auto hcols = [&](auto kern) {
      constexpr int WGH = S::T * 2;
      const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + 2 * S::PADDED * 8 + kHalfHL * WGH * 16;
      return std::function<hipError_t()>([=] {
        int grid = persistent_grid(kern, WGH, lds, fp.cascades * HalfCfg<11>::STRIPS * 2, cus);
        const int slices = cus * (1024 / WGH);
        grid = grid > slices ? slices : grid;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(WGH), lds, 0, fp, h02, gab, gcd, ge, tw, hs, HalfSlab{},
                           reinterpret_cast<unsigned char*>(spec), 1, nullptr);
        return hipGetLastError();
      });
    };
    auto hrows = [&](auto kern, int rpw) {
      const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + lds_row_slots<11>(rpw) * 8;
      return std::function<hipError_t()>([=] {
        const int grid = persistent_grid(kern, S::T * rpw, lds, fp.cascades * (n / rpw), cus);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(S::T * rpw), lds, 0, fp, gab, gcd, ge, spec, maps, jac, foam, tw, n,
                           RowSrc{}, (const float2*)nullptr);
        return hipGetLastError();
      });
    };
#define KH2(HK) k_cols_half<11, kStream, kStream, true, false, false, kHalfRG2, kHalfRGC2, 2, true, false, kHalfHL, HK, 0, 2, false, 2, 0, true>
    std::vector<std::function<hipError_t()>> vc = {prod_c, hcols(KH2(2)), hcols(KH2(4)), hcols(KH2(2)), hcols(KH2(2))};
    std::vector<std::function<hipError_t()>> vr = {prod_r,
                                                   hrows(k_rows_half<11, 0, kStream, 0, 2, true, false, kHalfRG2, kHalfRGC2, 2, 2>, 2),
                                                   hrows(k_rows_half<11, 0, kStream, 0, 2, true, false, kHalfRG2, kHalfRGC2, 2, 2>, 2),
                                                   hrows(k_rows_half<11, 0, kStream, 0, 2, true, false, kHalfRG2, kHalfRGC2, 2, 4>, 2),
                                                   hrows(k_rows_half<11, 0, kStream, 0, 1, true, false, kHalfRG2, kHalfRGC2, 2, 8>, 1)};
#undef KH2
    const char* nm[] = {"production (whole strips, FB 4)", "half strips HK 2 (FB 2)", "half strips HK 4 (FB 2)",
                        "HK 2, rows grouped 4 (FB 2)", "HK 2, one-row items grouped 8"};
    const int NV = 5;
    CHECK(vc[0]());
    CHECK(vr[0]());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb), pj = snap(jac, jb);
    std::vector<int> same(NV, 1);
    for (int k = 1; k < NV; k++)
    {
      CHECK(hipMemset(maps, 0, mb));
      CHECK(hipMemset(jac, 0, jb));
      CHECK(vc[k]());
      CHECK(vr[k]());
      CHECK(hipDeviceSynchronize());
      std::printf("%s vs production: maps, jacobian\n", nm[k]);
      same[k] = (int)diff(snap(maps, mb), pm) & (int)diff(snap(jac, jb), pj);
    }
    std::vector<std::vector<float>> tc(NV), tr(NV), tf(NV);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < NV; k++)
      {
        tc[k].push_back(time_ms(vc[k], 20));
        tr[k].push_back(time_ms(vr[k], 20));
        tf[k].push_back(time_ms([&] { CHECK(vc[k]()); return vr[k](); }, 20));
      }
    for (int k = 0; k < NV; k++)
    {
      std::sort(tc[k].begin(), tc[k].end());
      std::sort(tr[k].begin(), tr[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("%-34s cols %7.4f ms  rows %7.4f ms  frame %7.4f ms  bit-identical %s\n", nm[k], tc[k][4], tr[k][4],
                  tf[k][4], same[k] ? "yes" : "NO");
    }
    CHECK(hipFree(h02));
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "tail") == 0 && logn <= 12)
  {
    // round 6: is the one-cascade column pass bound by the one CU that holds two items? The strip-dealt
    // column pass (one rank) over the first ns strips, ns = STRIPS (the whole grid: N/8 + 1 items for
    // 256 CUs at 2048) down to fewer: timing only (the Nyquist-row term kernel included in every line)
    const int S0 = HalfCfg<11>::STRIPS;
    const int strips_all = logn == 11 ? S0 : logn == 12 ? HalfCfg<12>::STRIPS : HalfCfg<10>::STRIPS;
    unsigned char* send;
    const HalfSlab full{0, strips_all, strips_all, n};
    CHECK(hipMalloc(&send, half_slab_block_bytes(logn, C, full)));
    std::vector<int> counts = {strips_all, strips_all - 1, strips_all - 2, strips_all - 8, strips_all - 32,
                               (strips_all - 1) / 2 + 1, (strips_all - 1) / 2};
    for (int ns : counts)
    {
      const HalfSlab h{0, ns, strips_all, n};
      auto run = [&] {
        return launch_half_slab_columns(logn, fp, h, 1, h0, true, nullptr, send, tw, 0, cus, hs, cus, nullptr);
      };
      std::vector<float> t;
      for (int r = 0; r < 9; r++)
        t.push_back(time_ms(run, 20));
      std::sort(t.begin(), t.end());
      std::printf("strip-dealt column pass, N %d, %4d strips: median %7.4f ms\n", n, ns, t[4]);
    }
    CHECK(hipFree(send));
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "hp1") == 0 && logn == 12 && C <= 2)
  {
    // round 6: the row pass at <= 2 cascades (FB = 2 fields of the half-strip column pass) with the next
    // image's loads before the stores (EARLY) and three or four workgroups per CU (MINB), against
    // production (EARLY 0, MINB 4); maps bit-identical, medians of 9 x 20 launches
    using S = FftShape<12>;
    float4* h02;
    CHECK(hipMalloc(&h02, tex * C * sizeof(float4)));
    for (int c = 0; c < C; c++)
    {
      OceanSettings st{};
      st.seed[0] = 12342; st.seed[1] = 8934; st.U_10 = 40; st.theta_0 = 25; st.F = 800000; st.g = 9.8f;
      st.swell = 0.5f; st.h = 100; st.displacement = 0.4f; st.planeSize = planes[c % 8]; st.scale = 1; st.spread = 0.2f;
      CHECK(launch_generate_spectrum(st, n, h02 + tex * c, 0, cus, 0, 0, 2));
    }
    auto cols = [&] { return launch_half_columns(logn, fp, h02, gab, gcd, ge, spec, tw, 0, cus, hs, cus); };
    (void)sizeof(S);
    auto rows = [&](auto kern) {
      return std::function<hipError_t()>([=] {
        const int grid = persistent_grid(kern, 256, HpCfg::LDS, fp.cascades * n, cus);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), HpCfg::LDS, 0, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0,
                           RowSrc{});
        return hipGetLastError();
      });
    };
    std::vector<std::function<hipError_t()>> vr = {
        [&] { return launch_half_rows(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus); },
        rows(k_rows_hp<kHalfRG2, kHalfRGC2, false, false, 2, kHalfRGC2, 1, 4>),
        rows(k_rows_hp<kHalfRG2, kHalfRGC2, false, false, 2, kHalfRGC2, 1, 3>),
        rows(k_rows_hp<kHalfRG2, kHalfRGC2, false, false, 2, kHalfRGC2, 2, 3>),
        rows(k_rows_hp<kHalfRG2, kHalfRGC2, false, false, 2, kHalfRGC2, 0, 3>)};
    const char* nm[] = {"production (EARLY 0, 4 WG/CU)", "EARLY 1, 4 WG/CU", "EARLY 1, 3 WG/CU", "EARLY 2, 3 WG/CU",
                        "EARLY 0, 3 WG/CU"};
    const int NV = 5;
    CHECK(cols());
    CHECK(vr[0]());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb), pj = snap(jac, jb);
    std::vector<int> same(NV, 1);
    for (int k = 1; k < NV; k++)
    {
      CHECK(hipMemset(maps, 0, mb));
      CHECK(hipMemset(jac, 0, jb));
      CHECK(vr[k]());
      CHECK(hipDeviceSynchronize());
      std::printf("%s vs production: maps, jacobian\n", nm[k]);
      same[k] = (int)diff(snap(maps, mb), pm) & (int)diff(snap(jac, jb), pj);
    }
    std::vector<std::vector<float>> t(NV), tf(NV);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < NV; k++)
      {
        t[k].push_back(time_ms(vr[k], 20));
        tf[k].push_back(time_ms([&] { CHECK(cols()); return vr[k](); }, 20));
      }
    for (int k = 0; k < NV; k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("rows %-32s median %7.4f ms   frame %7.4f ms  bit-identical %s\n", nm[k], t[k][4], tf[k][4],
                  same[k] ? "yes" : "NO");
    }
    CHECK(hipFree(h02));
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "qxh") == 0 && logn == 12 && C <= 2)
  {
    // round 6: the half-strip column pass (<= 2 cascades: 512-thread workgroups, two per CU, FB = 2
    // fields, 2-column h0 strips) with quarter LDS exchanges so all 8 H pairs stay on the CU, against
    // production; frame = + the production row pass (launch_half_rows reads the FB = 2 layout)
    using S = FftShape<12>;
    float4* h02;  // h0 in 2-column strips (half_h0_block): what the production half-strip pass reads
    CHECK(hipMalloc(&h02, tex * C * sizeof(float4)));
    for (int c = 0; c < C; c++)
    {
      OceanSettings st{};
      st.seed[0] = 12342; st.seed[1] = 8934; st.U_10 = 40; st.theta_0 = 25; st.F = 800000; st.g = 9.8f;
      st.swell = 0.5f; st.h = 100; st.displacement = 0.4f; st.planeSize = planes[c % 8]; st.scale = 1; st.spread = 0.2f;
      CHECK(launch_generate_spectrum(st, n, h02 + tex * c, 0, cus, 0, 0, 2));
    }
    auto cols = [&](auto kern, int hl, bool qx) {
      const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + 2 * S::PADDED * (qx ? 4 : 8) + hl * 512 * 16;
      return std::function<hipError_t()>([=] {
        int grid = persistent_grid(kern, 512, lds, fp.cascades * HalfCfg<12>::STRIPS * 2, cus);
        grid = grid > 2 * cus ? 2 * cus : grid;  // hs: cus slices of 16 x 1024 entries = 2 cus half slices
        hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, 0, fp, h02, gab, gcd, ge, tw, hs, HalfSlab{},
                           (unsigned char*)spec, 1, nullptr);
        return hipGetLastError();
      });
    };
#define KQH(HL, HK, QX) k_cols_half<12, kStream, kStream, true, false, false, kHalfRG2, kHalfRGC2, 2, true, false, HL, HK, 0, 2, false, 2, 0, true, QX>
    std::vector<std::function<hipError_t()>> vc = {cols(KQH(1, 4, false), 1, false), cols(KQH(5, 3, true), 5, true),
                                                   cols(KQH(4, 4, true), 4, true), cols(KQH(1, 4, true), 1, true)};
#undef KQH
    const char* nm[] = {"production half strips (HL1 HK4)", "QX HL5 HK3 (no scratch)", "QX HL4 HK4 (no scratch)",
                        "QX HL1 HK4"};
    const int NV = 4;
    auto rows = [&] { return launch_half_rows(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus); };
    CHECK(vc[0]());
    CHECK(hipDeviceSynchronize());
    auto pab = snap(gab, ht * sizeof(float4)), pde = snap(gcd, ht * sizeof(float4)), pc = snap(ge, ht * sizeof(float2));
    std::vector<int> same(NV, 1);
    for (int k = 1; k < NV; k++)
    {
      CHECK(hipMemset(gab, 0, ht * sizeof(float4)));
      CHECK(hipMemset(gcd, 0, ht * sizeof(float4)));
      CHECK(hipMemset(ge, 0, ht * sizeof(float2)));
      CHECK(vc[k]());
      CHECK(hipDeviceSynchronize());
      std::printf("%s vs production: gab, gde, gc\n", nm[k]);
      same[k] = (int)diff(snap(gab, ht * sizeof(float4)), pab) & (int)diff(snap(gcd, ht * sizeof(float4)), pde) &
                (int)diff(snap(ge, ht * sizeof(float2)), pc);
    }
    std::vector<std::vector<float>> t(NV), tf(NV);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < NV; k++)
      {
        t[k].push_back(time_ms(vc[k], 20));
        tf[k].push_back(time_ms([&] { CHECK(vc[k]()); return rows(); }, 20));
      }
    for (int k = 0; k < NV; k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("cols %-34s median %7.4f ms   frame %7.4f ms  bit-identical %s\n", nm[k], t[k][4], tf[k][4],
                  same[k] ? "yes" : "NO");
    }
    CHECK(hipFree(h02));
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "oneshot") == 0 && logn == 12)
  {
    // round 6: the whole-strip column pass on a one-shot grid (one workgroup per item, handed out in
    // order by the dispatcher; the H scratch then needs one slice per item) against the production
    // persistent grid of one workgroup per CU; fields bit-identical (same arithmetic per item)
    using S = FftShape<12>;
    const int items = fp.cascades * HalfCfg<12>::STRIPS;
    float2* hsx;
    CHECK(hipMalloc(&hsx, (size_t)items * 16 * 1024 * sizeof(float2)));
    const int ldsw = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + ColFirstCfg<12>::LDS1 + kHalfHL * 1024 * 16;
    auto kern = k_cols_half<12, kStream, kStream, true, false, false, kHalfRG, kHalfRGC, 4, true, false, kHalfHL, kHalfHK, 0, 4,
                            false, 4, 0, true>;
    auto run = [&](int grid, float2* scratch) {
      return std::function<hipError_t()>([=] {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(1024), ldsw, 0, fp, h0, gab, gcd, ge, tw, scratch, HalfSlab{},
                           (unsigned char*)spec, 1, nullptr);
        return hipGetLastError();
      });
    };
    std::vector<std::function<hipError_t()>> vc = {run(cus, hs), run(items, hsx), run(2 * cus, hsx), run(4 * cus, hsx)};
    const char* nm[] = {"persistent, 1 per CU (production)", "one-shot (one workgroup per item)", "persistent, 2 x CUs",
                        "persistent, 4 x CUs"};
    const int NV = 4;
    CHECK(vc[0]());
    CHECK(hipDeviceSynchronize());
    auto pab = snap(gab, ht * sizeof(float4)), pde = snap(gcd, ht * sizeof(float4)), pc = snap(ge, ht * sizeof(float2));
    std::vector<int> same(NV, 1);
    for (int k = 1; k < NV; k++)
    {
      CHECK(hipMemset(gab, 0, ht * sizeof(float4)));
      CHECK(hipMemset(gcd, 0, ht * sizeof(float4)));
      CHECK(hipMemset(ge, 0, ht * sizeof(float2)));
      CHECK(vc[k]());
      CHECK(hipDeviceSynchronize());
      std::printf("%s vs production: gab, gde, gc\n", nm[k]);
      same[k] = (int)diff(snap(gab, ht * sizeof(float4)), pab) & (int)diff(snap(gcd, ht * sizeof(float4)), pde) &
                (int)diff(snap(ge, ht * sizeof(float2)), pc);
    }
    std::vector<std::vector<float>> t(NV), tf(NV);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < NV; k++)
      {
        t[k].push_back(time_ms(vc[k], 10));
        tf[k].push_back(time_ms([&] { CHECK(vc[k]()); return r1(); }, 10));
      }
    for (int k = 0; k < NV; k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("cols %-36s median %7.4f ms (%6.1f GB/s at 28.05 B/pt)  frame %7.4f ms  bit-identical %s\n", nm[k],
                  t[k][4], 28.05 * pts / t[k][4] / 1e6, tf[k][4], same[k] ? "yes" : "NO");
    }
    CHECK(hipFree(hsx));
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "hs4d") == 0 && logn == 12)
  {
    // round 6: half-strip pass 1 (two 512-thread workgroups per CU, 2-column h0 strips) into the whole
    // strips' 4-column fields, each 128-B field line written as two 64-B halves by the two items of a
    // strip (paired on one XCD), with DEFAULT-policy stores so that L2 merges the halves before writing
    // the line back; round 5's hs4 measured this layout with streamed (nt) stores: 2.48 ms. Frames with
    // the production whole-strip row pass (k_rows_hp FB 4, three per CU, EARLY 1; four per CU at <= 2
    // cascades); at <= 2 cascades also the production half-strip shape (FB 2). Maps vs production.
    using K = ColFirstCfg<12>;
    using S = FftShape<12>;
    float4* h0b2;
    CHECK(hipMalloc(&h0b2, tex * C * sizeof(float4)));
    for (int c = 0; c < C; c++)
    {
      OceanSettings st{};
      st.seed[0] = 12342; st.seed[1] = 8934; st.U_10 = 40; st.theta_0 = 25; st.F = 800000; st.g = 9.8f;
      st.swell = 0.5f; st.h = 100; st.displacement = 0.4f; st.planeSize = planes[c % 8]; st.scale = 1; st.spread = 0.2f;
      CHECK(launch_generate_spectrum(st, n, h0b2 + tex * c, 0, cus, 0, 0, 2));
    }
    const int tw0 = ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
    const int lds4 = tw0 + K::LDS1 + kHalfHL * 1024 * 16, lds2 = tw0 + 2 * S::PADDED * 8 + kHalfHL * 512 * 16;
    auto cols = [&](auto kern, int wg, int lds, const float4* hsrc) {
      return std::function<hipError_t()>([=] {
        const int items = fp.cascades * HalfCfg<12>::STRIPS * (K::WG1 / wg);
        int grid = persistent_grid(kern, wg, lds, items, cus);
        const int slices = cus * (1024 / wg);
        grid = grid > slices ? slices : grid;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(wg), lds, 0, fp, hsrc, gab, gcd, ge, tw, hs, HalfSlab{},
                           (unsigned char*)spec, 1, nullptr);
        return hipGetLastError();
      });
    };
    auto rows4 = [&] {
      auto kern = C <= 2 ? k_rows_hp<kHalfRG, kHalfRGC> : k_rows_hp<kHalfRG, kHalfRGC, false, false, 4, 4, 1, 3>;
      const int grid = persistent_grid(kern, 256, HpCfg::LDS, fp.cascades * n, cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), HpCfg::LDS, 0, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, RowSrc{});
      return hipGetLastError();
    };
    auto prod_cols = [&] { return launch_half_columns(logn, fp, C <= 2 ? h0b2 : h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus, nullptr, C <= 2 ? 2 : 0); };
    auto prod_rows = [&] { return launch_half_rows(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus); };
    std::vector<std::function<hipError_t()>> vc = {
        cols(k_cols_half<12, kStream, kStream, true, false, false, kHalfRG, kHalfRGC, 4, true, false, kHalfHL, kHalfHK, 0, 4, false, 4, 0, true>, 1024, lds4, h0),
        cols(k_cols_half<12, kStream, kStream, true, false, false, kHalfRG, kHalfRGC, 2, true, false, kHalfHL, 4, 0, 4, false, 2, 0, true>, 512, lds2, h0b2),
        cols(k_cols_half<12, kStream, 0, true, false, false, kHalfRG, kHalfRGC, 2, true, false, kHalfHL, 4, 0, 4, false, 2, 0, true>, 512, lds2, h0b2)};
    std::vector<std::function<hipError_t()>> vr = {rows4, rows4, rows4};
    std::vector<const char*> nm = {"whole strips (FB 4)", "half strips -> FB 4, nt stores", "half strips -> FB 4, default stores"};
    if (C <= 2)
    {
      vc.push_back(prod_cols);
      vr.push_back(prod_rows);
      nm.push_back("production at <= 2 (FB 2)");
    }
    const int NV = (int)vc.size();
    CHECK(vc[0]());
    CHECK(vr[0]());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb), pj = snap(jac, jb);
    std::vector<int> same(NV, 1);
    for (int k = 1; k < NV; k++)
    {
      CHECK(hipMemset(maps, 0, mb));
      CHECK(hipMemset(jac, 0, jb));
      CHECK(vc[k]());
      CHECK(vr[k]());
      CHECK(hipDeviceSynchronize());
      std::printf("%s vs whole strips: maps, jacobian\n", nm[k]);
      same[k] = (int)diff(snap(maps, mb), pm) & (int)diff(snap(jac, jb), pj);
    }
    std::vector<std::vector<float>> t(NV), tr(NV), tf(NV);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < NV; k++)
      {
        t[k].push_back(time_ms(vc[k], 10));
        tr[k].push_back(time_ms(vr[k], 10));
        tf[k].push_back(time_ms([&] { CHECK(vc[k]()); return vr[k](); }, 10));
      }
    for (int k = 0; k < NV; k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::sort(tr[k].begin(), tr[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("C=%d %-38s cols %7.4f  rows %7.4f  frame %7.4f ms  maps bit-identical %s\n", C, nm[k], t[k][4],
                  tr[k][4], tf[k][4], same[k] ? "yes" : "NO");
    }
    CHECK(hipFree(h0b2));
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "small") == 0 && logn <= 11)
  {
    // round 6: the small-grid column pass (k_cols_small: 8 points per thread, radix-8 Stockham, H in
    // VGPRs, N / 8 threads per column) against production k_cols_half; frame = + the production row
    // pass. The fields differ by FFT rounding only: max |diff| / max |field| is printed per field.
    auto prod = [&] { return launch_half_columns(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus); };
    auto rows = [&] { return launch_half_rows(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus); };
    std::function<hipError_t()> small;
    auto mk = [&](auto L) {
      constexpr int LG = decltype(L)::value;
      using CS = ColsSmallCfg<LG>;
      auto kern = k_cols_small<LG, kHalfRG, kHalfRGC>;
      small = [=] {
        const int grid = persistent_grid(kern, CS::WG, CS::LDS, fp.cascades * HalfCfg<LG>::STRIPS, cus);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(CS::WG), CS::LDS, 0, fp, h0, gab, gcd, ge, tw, spec);
        return hipGetLastError();
      };
    };
    if (logn == 10)
      mk(std::integral_constant<int, 10>{});
    else
      mk(std::integral_constant<int, 11>{});
    auto rel = [](const std::vector<unsigned char>& a, const std::vector<unsigned char>& b) {
      const float* x = reinterpret_cast<const float*>(a.data());
      const float* y = reinterpret_cast<const float*>(b.data());
      double mx = 0, er = 0;
      for (size_t k = 0; k < a.size() / 4; k++)
      {
        mx = std::max(mx, (double)std::fabs(x[k]));
        er = std::max(er, (double)std::fabs(x[k] - y[k]));
      }
      return er / (mx > 0 ? mx : 1);
    };
    CHECK(prod());
    CHECK(hipDeviceSynchronize());
    auto pab = snap(gab, ht * sizeof(float4)), pde = snap(gcd, ht * sizeof(float4)), pc = snap(ge, ht * sizeof(float2));
    auto psp = snap(spec, (size_t)C * 2 * n * sizeof(float4));
    CHECK(rows());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb);
    CHECK(hipMemset(gab, 0, ht * sizeof(float4)));
    CHECK(hipMemset(gcd, 0, ht * sizeof(float4)));
    CHECK(hipMemset(ge, 0, ht * sizeof(float2)));
    CHECK(hipMemset(spec, 0, (size_t)C * 2 * n * sizeof(float4)));
    CHECK(small());
    CHECK(hipDeviceSynchronize());
    std::printf("k_cols_small vs production, max |diff| / max: gab %.3g  gde %.3g  gc %.3g  spec %.3g\n",
                rel(pab, snap(gab, ht * sizeof(float4))), rel(pde, snap(gcd, ht * sizeof(float4))),
                rel(pc, snap(ge, ht * sizeof(float2))), rel(psp, snap(spec, (size_t)C * 2 * n * sizeof(float4))));
    CHECK(rows());
    CHECK(hipDeviceSynchronize());
    std::printf("maps from k_cols_small's fields vs production: max |diff| / max %.3g\n", rel(pm, snap(maps, mb)));
    std::vector<std::function<hipError_t()>> vc = {prod, small};
    const char* nm[] = {"production k_cols_half", "k_cols_small (8 points/thread)"};
    std::vector<std::vector<float>> t(2), tf(2);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < 2; k++)
      {
        t[k].push_back(time_ms(vc[k], 50));
        tf[k].push_back(time_ms([&] { CHECK(vc[k]()); return rows(); }, 50));
      }
    for (int k = 0; k < 2; k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("N=%d C=%d cols %-32s median %7.4f ms   frame %7.4f ms (%5.3f of 8 TB/s at 84 B/pt)\n", n, C, nm[k],
                  t[k][4], tf[k][4], 84.19 * pts / tf[k][4] / 1e6 / 8000.0);
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "rsplit") == 0)
  {
    // round 6: one workgroup per (strip, field round) on a one-shot grid (k_cols_half RSPLIT: h0
    // re-read and H re-evolved per round, the three slots of a strip on one XCD) against production;
    // frame = + the production row pass. For the latency-bound small grids (BASELINE config 3: 2048^2,
    // one cascade). Fields bit-identical (the same evolve and transform per round).
    auto prod = [&] { return launch_half_columns(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus); };
    auto rows = [&] { return launch_half_rows(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus); };
    auto rsplit = [&](auto L, auto kern) {
      constexpr int LG = decltype(L)::value;
      using K = ColFirstCfg<LG>;
      using S = FftShape<LG>;
      const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + K::LDS1;
      return std::function<hipError_t()>([=] {
        const int slots = fp.cascades * HalfCfg<LG>::STRIPS * 3;
        const int grid = (slots + 23) / 24 * 24;
        (void)persistent_grid(kern, K::WG1, lds, slots, cus);  // sets the dynamic-LDS attribute
        hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG1), lds, 0, fp, h0, gab, gcd, ge, tw, (float2*)nullptr, HalfSlab{},
                           (unsigned char*)spec, 1, nullptr);
        return hipGetLastError();
      });
    };
    std::vector<std::function<hipError_t()>> vc = {prod};
    auto add = [&](auto L) {
      constexpr int LG = decltype(L)::value;
      using K = ColFirstCfg<LG>;
      vc.push_back(rsplit(L, k_cols_half<LG, 0, kStream, false, false, false, kHalfRG, kHalfRGC, K::B, false, false, 0, 0, 0,
                                         4, false, K::B, 0, true, false, 0, true>));
      vc.push_back(rsplit(L, k_cols_half<LG, kStream, kStream, false, false, false, kHalfRG, kHalfRGC, K::B, false, false, 0,
                                         0, 0, 4, false, K::B, 0, true, false, 0, true>));
    };
    if (logn == 10)
      add(std::integral_constant<int, 10>{});
    else if (logn == 11)
      add(std::integral_constant<int, 11>{});
    else
      add(std::integral_constant<int, 12>{});
    const char* nm[] = {"production", "RSPLIT, h0 default policy", "RSPLIT, h0 streamed"};
    const int NV = 3;
    CHECK(vc[0]());
    CHECK(hipDeviceSynchronize());
    auto pab = snap(gab, ht * sizeof(float4)), pde = snap(gcd, ht * sizeof(float4)), pc = snap(ge, ht * sizeof(float2));
    std::vector<int> same(NV, 1);
    for (int k = 1; k < NV; k++)
    {
      CHECK(hipMemset(gab, 0, ht * sizeof(float4)));
      CHECK(hipMemset(gcd, 0, ht * sizeof(float4)));
      CHECK(hipMemset(ge, 0, ht * sizeof(float2)));
      CHECK(vc[k]());
      CHECK(hipDeviceSynchronize());
      std::printf("%s vs production: gab, gde, gc\n", nm[k]);
      same[k] = (int)diff(snap(gab, ht * sizeof(float4)), pab) & (int)diff(snap(gcd, ht * sizeof(float4)), pde) &
                (int)diff(snap(ge, ht * sizeof(float2)), pc);
    }
    std::vector<std::vector<float>> t(NV), tf(NV);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < NV; k++)
      {
        t[k].push_back(time_ms(vc[k], 50));
        tf[k].push_back(time_ms([&] { CHECK(vc[k]()); return rows(); }, 50));
      }
    std::printf("N=%d cascades=%d, rows alone %7.4f ms\n", n, C, time_ms(rows, 50));
    for (int k = 0; k < NV; k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("cols %-28s median %7.4f ms   frame %7.4f ms (%5.3f of 8 TB/s at 84 B/pt)  bit-identical %s\n", nm[k],
                  t[k][4], tf[k][4], 84.19 * pts / tf[k][4] / 1e6 / 8000.0, same[k] ? "yes" : "NO");
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "desync") == 0 && logn == 12)
  {
    // round 6: half-strip column pass (512-thread workgroups, two per CU, FB = 2 fields, 2-column h0
    // strips) at any cascade count, with the second half of the grid starting DELAY ticks late so the two
    // workgroups of a CU store out of step; against the whole-strip production pass. Frames: + the row
    // pass of each layout (k_rows_hp FB = 4 three per CU / FB = 2 four per CU). Fields compared per layout.
    using S = FftShape<12>;
    float4* h02;
    CHECK(hipMalloc(&h02, tex * C * sizeof(float4)));
    for (int c = 0; c < C; c++)
    {
      OceanSettings st{};
      st.seed[0] = 12342; st.seed[1] = 8934; st.U_10 = 40; st.theta_0 = 25; st.F = 800000; st.g = 9.8f;
      st.swell = 0.5f; st.h = 100; st.displacement = 0.4f; st.planeSize = planes[c % 8]; st.scale = 1; st.spread = 0.2f;
      CHECK(launch_generate_spectrum(st, n, h02 + tex * c, 0, cus, 0, 0, 2));
    }
    const int ldsw = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + ColFirstCfg<12>::LDS1 + kHalfHL * 1024 * 16;
    const int ldsh = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + 2 * S::PADDED * 8 + kHalfHL * 512 * 16;
    auto whole = [&] {
      auto kern = k_cols_half<12, kStream, kStream, true, false, false, kHalfRG, kHalfRGC, 4, true, false, kHalfHL, kHalfHK, 0, 4,
                              false, 4, 0, true>;
      int grid = persistent_grid(kern, 1024, ldsw, fp.cascades * HalfCfg<12>::STRIPS, cus);
      grid = grid > cus ? cus : grid;
      hipLaunchKernelGGL(kern, dim3(grid), dim3(1024), ldsw, 0, fp, h0, gab, gcd, ge, tw, hs, HalfSlab{}, (unsigned char*)spec,
                         1, nullptr);
      return hipGetLastError();
    };
    auto half = [&](auto kern, bool resident) {
      return std::function<hipError_t()>([=] {
        int grid = resident ? 2 * cus : persistent_grid(kern, 512, ldsh, fp.cascades * HalfCfg<12>::STRIPS * 2, cus);
        grid = grid > 2 * cus ? 2 * cus : grid;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(512), ldsh, 0, fp, h02, gab, gcd, ge, tw, hs, HalfSlab{},
                           (unsigned char*)spec, 1, nullptr);
        return hipGetLastError();
      });
    };
#define KD(D) k_cols_half<12, kStream, kStream, true, false, false, kHalfRG2, kHalfRGC2, 2, true, false, kHalfHL, kHalfHK, 0, 2, false, 2, 0, true, false, D>
    std::vector<std::function<hipError_t()>> vc = {whole, half(KD(0), false), half(KD(0), true), half(KD(400), true),
                                                   half(KD(800), true), half(KD(1600), true)};
#undef KD
    const char* nm[] = {"whole strips (production >= 3)", "half strips", "half strips, resident grid",
                        "half, resident, delay 4 us", "half, resident, delay 8 us", "half, resident, delay 16 us"};
    const int NV = 6;
    auto rows4 = [&] {
      auto kern = k_rows_hp<kHalfRG, kHalfRGC, false, false, 4, 4, 1, 3>;
      const int grid = persistent_grid(kern, 256, HpCfg::LDS, fp.cascades * n, cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), HpCfg::LDS, 0, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, RowSrc{});
      return hipGetLastError();
    };
    auto rows2 = [&] {
      auto kern = k_rows_hp<kHalfRG2, kHalfRGC2, false, false, 2, kHalfRGC2>;
      const int grid = persistent_grid(kern, 256, HpCfg::LDS, fp.cascades * n, cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), HpCfg::LDS, 0, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, RowSrc{});
      return hipGetLastError();
    };
    CHECK(vc[0]());
    CHECK(rows4());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb), pj = snap(jac, jb);
    std::vector<int> same(NV, 1);
    for (int k = 1; k < NV; k++)
    {
      CHECK(hipMemset(maps, 0, mb));
      CHECK(hipMemset(jac, 0, jb));
      CHECK(vc[k]());
      CHECK(rows2());
      CHECK(hipDeviceSynchronize());
      std::printf("%s vs whole strips: maps, jacobian\n", nm[k]);
      same[k] = (int)diff(snap(maps, mb), pm) & (int)diff(snap(jac, jb), pj);
    }
    std::vector<std::vector<float>> t(NV), tf(NV);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < NV; k++)
      {
        t[k].push_back(time_ms(vc[k], 10));
        tf[k].push_back(time_ms([&] { CHECK(vc[k]()); return k == 0 ? rows4() : rows2(); }, 10));
      }
    for (int k = 0; k < NV; k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("cols %-34s median %7.4f ms   frame %7.4f ms  maps bit-identical %s\n", nm[k], t[k][4], tf[k][4],
                  same[k] ? "yes" : "NO");
    }
    CHECK(hipFree(h02));
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "hpe") == 0 && logn == 12)
  {
    // k_rows_hp with the next image's / row's loads issued before the stores (EARLY 1, 2) against
    // production on the production fields: maps bit-identical, medians of 9 x 10 launches
    CHECK(c1());
    CHECK(hipDeviceSynchronize());
    auto rows = [&](auto kern) {
      return std::function<hipError_t()>([=] {
        const int grid = persistent_grid(kern, 256, HpCfg::LDS, fp.cascades * n, cus);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), HpCfg::LDS, 0, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0,
                           RowSrc{});
        return hipGetLastError();
      });
    };
    std::vector<std::function<hipError_t()>> vr = {rows(k_rows_hp<kHalfRG, kHalfRGC>),
                                                   rows(k_rows_hp<kHalfRG, kHalfRGC, false, false, 4, 4, 1>),
                                                   rows(k_rows_hp<kHalfRG, kHalfRGC, false, false, 4, 4, 2>),
                                                   rows(k_rows_hp<kHalfRG, kHalfRGC, false, false, 4, 4, 0, 3>),
                                                   rows(k_rows_hp<kHalfRG, kHalfRGC, false, false, 4, 4, 2, 3>),
                                                   rows(k_rows_hp<kHalfRG, kHalfRGC, false, false, 4, 4, 1, 3>)};
    const char* nm[] = {"k_rows_hp (production)", "k_rows_hp EARLY 1", "k_rows_hp EARLY 2", "3 WG/CU",
                        "3 WG/CU EARLY 2", "3 WG/CU EARLY 1"};
    const int NV = 6;
    CHECK(vr[0]());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb), pj = snap(jac, jb);
    std::vector<int> same(NV, 1);
    for (int k = 1; k < NV; k++)
    {
      CHECK(hipMemset(maps, 0, mb));
      CHECK(hipMemset(jac, 0, jb));
      CHECK(vr[k]());
      CHECK(hipDeviceSynchronize());
      std::printf("%s vs production: maps, jacobian\n", nm[k]);
      same[k] = (int)diff(snap(maps, mb), pm) & (int)diff(snap(jac, jb), pj);
    }
    std::vector<std::vector<float>> t(NV), tf(NV);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < NV; k++)
      {
        t[k].push_back(time_ms(vr[k], 10));
        tf[k].push_back(time_ms([&] { CHECK(c1()); return vr[k](); }, 10));
      }
    for (int k = 0; k < NV; k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("%-24s rows median %7.3f ms (%7.1f GB/s at 56 B/pt)  frame %7.3f ms  bit-identical %s\n", nm[k], t[k][4],
                  56.04 * pts / t[k][4] / 1e6, tf[k][4], same[k] ? "yes" : "NO");
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "abl") == 0)
  {
    // the production pass 1 alone (built with -DOCEAN_ABLATE_H0LOAD / -DOCEAN_ABLATE_FSTORE: timing
    // ablations, wrong fields); median of 9 x 10 launches
    std::vector<float> t;
    for (int r = 0; r < 9; r++)
      t.push_back(time_ms(c1, 10));
    std::sort(t.begin(), t.end());
    std::printf("cols production pass 1 median %7.3f ms (min %7.3f)\n", t[4], t[0]);
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "hkeep") == 0)
  {
    // pass 1 with some H pairs outside the scratch (variants 25..31: HL pairs in LDS, HK in VGPRs)
    // against all pairs in the scratch; the frame with the production row pass
    constexpr int NV = 8;
    // variant 32 = round 2's earlier production (all 8 pairs in the scratch); production now = 30
    const int vs[NV] = {32, 25, 26, 27, 28, 29, 30, 31};
    const char* nm[NV] = {"8 pairs in scratch (variant 32)", "HL 1 HK 0", "HL 1 HK 1", "HL 1 HK 2", "HL 0 HK 2", "HL 1 HK 3",
                          "HL 1 HK 4", "HL 1 HK 5"};
    CHECK(c1());
    CHECK(hipDeviceSynchronize());
    auto pab = snap(gab, ht * sizeof(float4)), pde = snap(gcd, ht * sizeof(float4)), pc = snap(ge, ht * sizeof(float2));
    bool same[NV] = {true};
    for (int k = 1; k < NV; k++)
    {
      CHECK(hipMemset(gab, 0, ht * sizeof(float4)));
      CHECK(hipMemset(gcd, 0, ht * sizeof(float4)));
      CHECK(hipMemset(ge, 0, ht * sizeof(float2)));
      CHECK(launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus, nullptr, vs[k]));
      CHECK(hipDeviceSynchronize());
      std::printf("%s vs variant 32: gab, gde, gc\n", nm[k]);
      same[k] = (int)diff(snap(gab, ht * sizeof(float4)), pab) & (int)diff(snap(gcd, ht * sizeof(float4)), pde) &
                (int)diff(snap(ge, ht * sizeof(float2)), pc);
    }
    std::vector<std::vector<float>> t(NV), tf(NV);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < NV; k++)
      {
        auto ck = [&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus, nullptr, vs[k]); };
        t[k].push_back(time_ms(ck, 10));
        tf[k].push_back(time_ms([&] { CHECK(ck()); return r1(); }, 10));
      }
    for (int k = 0; k < NV; k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("cols %-32s median %7.3f ms   frame %7.3f ms  bit-identical %s\n", nm[k], t[k][4], tf[k][4],
                  same[k] ? "yes" : "NO");
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "rowabl") == 0)
  {
    // the production row pass and its timing ablations (wrong results by construction): 1 no HBM
    // loads, 2 no x transform, 3 no mirror exchange; built with -DOCEAN_ABLATE_BARRIER /
    // -DOCEAN_ABLATE_EXCHANGE (halfbench_nobar / _noxch) the exchanges lose their barriers / LDS
    CHECK(c1());
    CHECK(hipDeviceSynchronize());
    const char* nm[] = {"rows (production)", "ABL 1: no HBM loads", "ABL 2: no x transform", "ABL 3: no mirror exchange"};
    std::vector<std::vector<float>> tr(4);
    for (int r = 0; r < 7; r++)
      for (int a = 0; a < 4; a++)
        tr[a].push_back(time_ms([&] { return launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus, a); }, 10));
    for (int a = 0; a < 4; a++)
    {
      std::sort(tr[a].begin(), tr[a].end());
      std::printf("%-28s median %7.3f ms  %7.1f GB/s at 56 B/pt\n", nm[a], tr[a][3], 56.04 * pts / tr[a][3] / 1e6);
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "xframe") == 0)
  {
    // frames pipelined over two field slots: frame f+1's pass 1 (depends on h0 and t only) on
    // stream A beside frame f's pass 2 on stream B; pass 2 of every frame stays in order on B, so
    // the maps are written frame after frame as before. Against both passes per frame on one stream.
    float4 *gab2, *gcd2, *spec2;
    float2* ge2;
    CHECK(hipMalloc(&gab2, ht * sizeof(float4)));
    CHECK(hipMalloc(&gcd2, ht * sizeof(float4)));
    CHECK(hipMalloc(&ge2, ht * sizeof(float2)));
    CHECK(hipMalloc(&spec2, (size_t)C * 2 * n * sizeof(float4)));
    float4* sab[2] = {gab, gab2};
    float4* sde[2] = {gcd, gcd2};
    float2* sc[2] = {ge, ge2};
    float4* ssp[2] = {spec, spec2};
    hipStream_t sa, sb;
    CHECK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    hipEvent_t evc[2], evr[2], e0;
    for (int k = 0; k < 2; k++)
    {
      CHECK(hipEventCreateWithFlags(&evc[k], hipEventDisableTiming));
      CHECK(hipEventCreateWithFlags(&evr[k], hipEventDisableTiming));
      CHECK(hipEventRecord(evr[k], 0));
    }
    CHECK(hipEventCreateWithFlags(&e0, hipEventDisableTiming));
    const int F = 20;
    auto serial = [&] {
      for (int f = 0; f < F; f++)
      {
        CHECK(c1());
        CHECK(r1());
      }
      return hipSuccess;
    };
    auto piped = [&] {
      CHECK(hipEventRecord(e0, 0));
      CHECK(hipStreamWaitEvent(sa, e0, 0));
      CHECK(hipStreamWaitEvent(sb, e0, 0));
      for (int f = 0; f < F; f++)
      {
        const int s = f & 1;
        CHECK(hipStreamWaitEvent(sa, evr[s], 0));
        CHECK(launch_half_columns_ab(logn, fp, h0, sab[s], sde[s], sc[s], ssp[s], tw, sa, cus, hs, cus));
        CHECK(hipEventRecord(evc[s], sa));
        CHECK(hipStreamWaitEvent(sb, evc[s], 0));
        CHECK(launch_half_rows_ab(logn, fp, sab[s], sde[s], sc[s], ssp[s], maps, jac, foam, tw, sb, cus));
        CHECK(hipEventRecord(evr[s], sb));
      }
      CHECK(hipStreamWaitEvent(0, evr[(F - 1) & 1], 0));
      return hipSuccess;
    };
    CHECK(serial());
    CHECK(hipDeviceSynchronize());
    auto bm = snap(maps, mb), bj = snap(jac, jb);
    CHECK(hipMemset(maps, 0, mb));
    CHECK(piped());
    CHECK(hipDeviceSynchronize());
    std::printf("pipelined vs serial frames:\n");
    const bool same = (int)diff(snap(maps, mb), bm) & (int)diff(snap(jac, jb), bj);
    std::vector<float> ts, tp;
    for (int r = 0; r < 7; r++)
    {
      ts.push_back(time_ms(serial, 1) / F);
      tp.push_back(time_ms(piped, 1) / F);
    }
    std::sort(ts.begin(), ts.end());
    std::sort(tp.begin(), tp.end());
    std::printf("C=%d frame, both passes on one stream     median %7.3f ms (%d frames)\n", C, ts[3], F);
    std::printf("C=%d frame, pass 1 of f+1 beside pass 2 of f median %7.3f ms  bit-identical %s\n", C, tp[3],
                same ? "yes" : "NO");
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "fb2h") == 0 && logn == 12)
  {
    // pass 1 on half strips at two 512-thread workgroups per CU (k_cols_half CPI = 2, 128 VGPRs, a
    // 68-KiB exchange each) with fields FB = 2 columns wide (whole-line stores: gab / gde RG = 4, gc
    // RGC = 8 or 4), the row pass k_rows_hp on that layout; against production (whole strips, one
    // 1024-thread workgroup per CU). Same per-column arithmetic; the maps are compared to rounding.
    using K = ColFirstCfg<12>;
    using S = FftShape<12>;
    const int tw0 = ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
    auto cols = [&](auto kern, int wg, int lds) {
      return std::function<hipError_t()>([=] {
        hipError_t e = launch_half_nyquist(fp, n, K::B, h0, spec, nullptr, 1, 0, nullptr, 0, cus);
        if (e != hipSuccess)
          return e;
        const int items = fp.cascades * HalfCfg<12>::STRIPS * (K::WG1 / wg);
        int grid = persistent_grid(kern, wg, lds, items, cus);
        const int slices = cus * (1024 / wg);  // hs: cus slices of 16 x 1024 entries
        grid = grid > slices ? slices : grid;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(wg), lds, 0, fp, h0, gab, gcd, ge, tw, hs, HalfSlab{},
                           (unsigned char*)nullptr, 1, nullptr);
        return hipGetLastError();
      });
    };
    auto rows = [&](auto kern) {
      return std::function<hipError_t()>([=] {
        const int grid = persistent_grid(kern, 256, HpCfg::LDS, fp.cascades * n, cus);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), HpCfg::LDS, 0, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0,
                           RowSrc{});
        return hipGetLastError();
      });
    };
    const int lds4 = tw0 + K::LDS1 + kHalfHL * 1024 * 16, lds2 = tw0 + 2 * S::PADDED * 8 + kHalfHL * 512 * 16;
    std::vector<std::function<hipError_t()>> vc = {
        cols(k_cols_half<12, kStream, kStream, true, false, false, kHalfRG, kHalfRGC, 4, true, false, kHalfHL, kHalfHK>, 1024, lds4),
        cols(k_cols_half<12, kStream, kStream, true, false, false, 4, 8, 2, true, false, kHalfHL, 4, 0, 2>, 512, lds2),
        cols(k_cols_half<12, kStream, kStream, true, false, false, 4, 8, 2, true, false, kHalfHL, 2, 0, 2>, 512, lds2),
        cols(k_cols_half<12, kStream, kStream, true, false, false, 4, 4, 2, true, false, kHalfHL, 4, 0, 2>, 512, lds2),
        cols(k_cols_half<12, kStream, kStream, true, false, false, 4, 8, 2, true, false, kHalfHL, 4, 0, 2>, 512, lds2),
        cols(k_cols_half<12, kStream, kStream, true, false, false, 4, 8, 2, true, false, kHalfHL, 4, 0, 2>, 512, lds2)};
    std::vector<std::function<hipError_t()>> vr = {rows(k_rows_hp<kHalfRG, kHalfRGC>),
                                                   rows(k_rows_hp<4, 8, false, false, 2, 8>),
                                                   rows(k_rows_hp<4, 8, false, false, 2, 8>),
                                                   rows(k_rows_hp<4, 4, false, false, 2, 4>),
                                                   rows(k_rows_hp<4, 8, false, false, 2, 4>),
                                                   rows(k_rows_hp<4, 8, false, false, 2, 16>)};
    const char* nm[] = {"production (whole strips)", "half strips FB 2, RGC 8, HK 4", "half strips FB 2, RGC 8, HK 2",
                        "half strips FB 2, RGC 4, HK 4", "FB 2, RGC 8, rows GRP 4", "FB 2, RGC 8, rows GRP 16"};
    const int NV = 6;
    auto rel = [](const std::vector<unsigned char>& a, const std::vector<unsigned char>& b) {
      const float* x = reinterpret_cast<const float*>(a.data());
      const float* y = reinterpret_cast<const float*>(b.data());
      double d = 0, m = 0;
      for (size_t k = 0; k < a.size() / 4; k++)
      {
        d = std::max(d, (double)std::fabs(x[k] - y[k]));
        m = std::max(m, (double)std::fabs(x[k]));
      }
      return d / (m > 0 ? m : 1);
    };
    CHECK(vc[0]());
    CHECK(vr[0]());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb), pj = snap(jac, jb);
    for (int k = 1; k < NV; k++)
    {
      CHECK(hipMemset(maps, 0, mb));
      CHECK(hipMemset(jac, 0, jb));
      CHECK(vc[k]());
      CHECK(vr[k]());
      CHECK(hipDeviceSynchronize());
      std::printf("%s vs production: maps %.2g jacobian %.2g (max |diff| / max)\n", nm[k], rel(snap(maps, mb), pm),
                  rel(snap(jac, jb), pj));
    }
    std::vector<std::vector<float>> t(NV), tr(NV), tf(NV);
    for (int r = 0; r < 9; r++)
      for (int k = 0; k < NV; k++)
      {
        t[k].push_back(time_ms(vc[k], 10));
        tr[k].push_back(time_ms(vr[k], 10));
        tf[k].push_back(time_ms([&] { CHECK(vc[k]()); return vr[k](); }, 10));
      }
    for (int k = 0; k < NV; k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::sort(tr[k].begin(), tr[k].end());
      std::sort(tf[k].begin(), tf[k].end());
      std::printf("%-32s cols %7.3f ms  rows %7.3f ms  frame %7.3f ms\n", nm[k], t[k][4], tr[k][4], tf[k][4]);
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "xgrid") == 0)
  {
    // frame overlap with the production launchers (k_cols_half, k_rows_hp): frame f+1's column pass on
    // stream A beside frame f's row pass on stream B, the column pass's persistent grid limited to
    // `ccus` workgroups (1 per CU) so frame f's row pass keeps the other CUs. Against serial frames.
    float4 *gab2, *gcd2, *spec2;
    float2* ge2;
    CHECK(hipMalloc(&gab2, ht * sizeof(float4)));
    CHECK(hipMalloc(&gcd2, ht * sizeof(float4)));
    CHECK(hipMalloc(&ge2, ht * sizeof(float2)));
    CHECK(hipMalloc(&spec2, (size_t)C * 2 * n * sizeof(float4)));
    float4* sab[2] = {gab, gab2};
    float4* sde[2] = {gcd, gcd2};
    float2* sc[2] = {ge, ge2};
    float4* ssp[2] = {spec, spec2};
    hipStream_t sa, sb;
    CHECK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    hipEvent_t evc[2], evr[2], e0;
    for (int k = 0; k < 2; k++)
    {
      CHECK(hipEventCreateWithFlags(&evc[k], hipEventDisableTiming));
      CHECK(hipEventCreateWithFlags(&evr[k], hipEventDisableTiming));
      CHECK(hipEventRecord(evr[k], 0));
    }
    CHECK(hipEventCreateWithFlags(&e0, hipEventDisableTiming));
    const int F = 20;
    auto pc = [&](int s, hipStream_t st, int ccus) {
      return launch_half_columns(logn, fp, h0, sab[s], sde[s], sc[s], ssp[s], tw, st, ccus, hs, cus, nullptr);
    };
    auto pr = [&](int s, hipStream_t st, int rcus) {
      return launch_half_rows(logn, fp, sab[s], sde[s], sc[s], ssp[s], maps, jac, foam, tw, st, rcus);
    };
    auto serial = [&] {
      for (int f = 0; f < F; f++)
      {
        CHECK(pc(0, 0, cus));
        CHECK(pr(0, 0, cus));
      }
      return hipSuccess;
    };
    auto piped = [&](int ccus, int rcus) {
      CHECK(hipEventRecord(e0, 0));
      CHECK(hipStreamWaitEvent(sa, e0, 0));
      CHECK(hipStreamWaitEvent(sb, e0, 0));
      for (int f = 0; f < F; f++)
      {
        const int s = f & 1;
        CHECK(hipStreamWaitEvent(sa, evr[s], 0));
        CHECK(pc(s, sa, ccus));
        CHECK(hipEventRecord(evc[s], sa));
        CHECK(hipStreamWaitEvent(sb, evc[s], 0));
        CHECK(pr(s, sb, rcus));
        CHECK(hipEventRecord(evr[s], sb));
      }
      CHECK(hipStreamWaitEvent(0, evr[(F - 1) & 1], 0));
      return hipSuccess;
    };
    CHECK(serial());
    CHECK(hipDeviceSynchronize());
    auto bm = snap(maps, mb), bj = snap(jac, jb);
    // bal: the fewest workgroups that keep the full grid's number of item rounds (ceil(items / 256))
    const int items = C * HalfCfg<12>::STRIPS, rounds = (items + cus - 1) / cus, bal = (items + rounds - 1) / rounds;
    const int cc[] = {cus, bal, 224, 192, 128};
    const int NC = 5;
    bool same[NC];
    for (int k = 0; k < NC; k++)
    {
      CHECK(hipMemset(maps, 0, mb));
      CHECK(piped(cc[k], cus));
      CHECK(hipDeviceSynchronize());
      std::printf("pipelined (column grid %d) vs serial frames:\n", cc[k]);
      same[k] = (int)diff(snap(maps, mb), bm) & (int)diff(snap(jac, jb), bj);
    }
    std::vector<float> ts;
    std::vector<std::vector<float>> tp(NC), tcol(NC);
    for (int r = 0; r < 7; r++)
    {
      ts.push_back(time_ms(serial, 1) / F);
      for (int k = 0; k < NC; k++)
      {
        tp[k].push_back(time_ms([&] { return piped(cc[k], cus); }, 1) / F);
        tcol[k].push_back(time_ms([&] { return pc(0, 0, cc[k]); }, 10));
      }
    }
    std::sort(ts.begin(), ts.end());
    std::printf("C=%d frame, serial                                  median %7.3f ms (%d frames)\n", C, ts[3], F);
    for (int k = 0; k < NC; k++)
    {
      std::sort(tp[k].begin(), tp[k].end());
      std::sort(tcol[k].begin(), tcol[k].end());
      std::printf("C=%d frame, overlapped, column grid %3d             median %7.3f ms  (column pass alone %7.3f ms)  bit-identical %s\n",
                  C, cc[k], tp[k][3], tcol[k][3], same[k] ? "yes" : "NO");
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "overlap") == 0)
  {
    // cascade groups pipelined over two streams: pass 1 of group g+1 (VALU-bound) beside pass 2 of
    // group g (HBM-bound), against both passes over all cascades on one stream
    hipStream_t sa, sb;
    CHECK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(C + 2);
    for (auto& evt : ev)
      CHECK(hipEventCreateWithFlags(&evt, hipEventDisableTiming));
    const size_t ht1 = half_field_texels(logn);
    auto grouped = [&](int G) {
      const int per = C / G;
      CHECK(hipEventRecord(ev[C], 0));
      CHECK(hipStreamWaitEvent(sa, ev[C], 0));
      CHECK(hipStreamWaitEvent(sb, ev[C], 0));
      for (int g = 0; g < G; g++)
      {
        const int c0 = g * per;
        FrameParams f1{};
        f1.cascades = per;
        FoamParams o1{};
        for (int k = 0; k < per; k++)
        {
          f1.c[k] = fp.c[c0 + k];
          o1.displacement[k] = foam.displacement[c0 + k];
        }
        hipError_t e = launch_half_columns_ab(logn, f1, h0 + tex * c0, gab + ht1 * c0, gcd + ht1 * c0, ge + ht1 * c0,
                                           spec + (size_t)2 * n * c0, tw, sa, cus, hs, cus);
        if (e != hipSuccess)
          return e;
        CHECK(hipEventRecord(ev[g], sa));
        CHECK(hipStreamWaitEvent(sb, ev[g], 0));
        e = launch_half_rows_ab(logn, f1, gab + ht1 * c0, gcd + ht1 * c0, ge + ht1 * c0, spec + (size_t)2 * n * c0,
                             maps + tex * 2 * c0, jac + tex * c0, o1, tw, sb, cus);
        if (e != hipSuccess)
          return e;
      }
      CHECK(hipEventRecord(ev[C + 1], sb));
      CHECK(hipStreamWaitEvent(0, ev[C + 1], 0));
      CHECK(hipStreamWaitEvent(0, ev[G - 1], 0));
      return hipSuccess;
    };
    auto batched = [&] { hipError_t e = c1(); return e == hipSuccess ? r1() : e; };
    CHECK(batched());
    CHECK(hipDeviceSynchronize());
    auto bm = snap(maps, mb), bj = snap(jac, jb);
    std::vector<int> gs;
    for (int G = 2; G <= C; G *= 2)
      if (C % G == 0)
        gs.push_back(G);
    std::vector<bool> same(gs.size());
    for (size_t k = 0; k < gs.size(); k++)
    {
      CHECK(hipMemset(maps, 0, mb));
      CHECK(grouped(gs[k]));
      CHECK(hipDeviceSynchronize());
      std::printf("%d groups vs batched frame:\n", gs[k]);
      same[k] = (int)diff(snap(maps, mb), bm) & (int)diff(snap(jac, jb), bj);
    }
    std::vector<std::vector<float>> tm(1 + gs.size());
    for (int r = 0; r < 7; r++)
    {
      tm[0].push_back(time_ms(batched, 10));
      for (size_t k = 0; k < gs.size(); k++)
        tm[1 + k].push_back(time_ms([&] { return grouped(gs[k]); }, 10));
    }
    for (auto& t : tm)
      std::sort(t.begin(), t.end());
    std::printf("frame batched, one stream            median %7.3f ms\n", tm[0][3]);
    for (size_t k = 0; k < gs.size(); k++)
      std::printf("frame %d groups, pass 2 on stream 2   median %7.3f ms  bit-identical %s\n", gs[k], tm[1 + k][3],
                  same[k] ? "yes" : "NO");
    return 0;
  }
  if (mall)
  {
    // one cascade at a time (pass 1 then pass 2 per cascade: its 336 MB of fields may still sit in
    // the 256 MB Infinity Cache when pass 2 reads them) against both passes over all cascades
    const size_t ht1 = half_field_texels(logn);
    auto per_cascade = [&] {
      for (int c = 0; c < C; c++)
      {
        FrameParams f1{};
        f1.cascades = 1;
        f1.c[0] = fp.c[c];
        FoamParams o1{};
        o1.displacement[0] = foam.displacement[c];
        hipError_t e = launch_half_columns_ab(logn, f1, h0 + tex * c, gab + ht1 * c, gcd + ht1 * c, ge + ht1 * c,
                                           spec + (size_t)2 * n * c, tw, 0, cus, hs, cus);
        if (e == hipSuccess)
          e = launch_half_rows_ab(logn, f1, gab + ht1 * c, gcd + ht1 * c, ge + ht1 * c, spec + (size_t)2 * n * c,
                               maps + tex * 2 * c, jac + tex * c, o1, tw, 0, cus);
        if (e != hipSuccess)
          return e;
      }
      return hipSuccess;
    };
    auto batched = [&] { hipError_t e = c1(); return e == hipSuccess ? r1() : e; };
    CHECK(batched());
    CHECK(hipDeviceSynchronize());
    auto bm = snap(maps, mb), bj = snap(jac, jb);
    CHECK(hipMemset(maps, 0, mb));
    CHECK(per_cascade());
    CHECK(hipDeviceSynchronize());
    std::printf("per-cascade frame vs batched frame:\n");
    const bool same = (int)diff(snap(maps, mb), bm) & (int)diff(snap(jac, jb), bj);
    std::vector<std::vector<float>> tm(2);
    for (int r = 0; r < 7; r++)
    {
      tm[0].push_back(time_ms(batched, 10));
      tm[1].push_back(time_ms(per_cascade, 10));
    }
    for (int k = 0; k < 2; k++)
      std::sort(tm[k].begin(), tm[k].end());
    std::printf("frame batched (2 launches)          median %7.3f ms\n", tm[0][3]);
    std::printf("frame per cascade (2 x %d launches) median %7.3f ms  bit-identical %s\n", C, tm[1][3], same ? "yes" : "NO");
    return 0;
  }
  {
    // pass 1 on half-strip items (k_cols_half CPI = B / 2, 512 threads, two workgroups per CU,
    // variant 20) against production (whole strips, 1024 threads, one per CU): fields must be
    // bit-identical (same per-column arithmetic), then timing of the pass and the frame
    CHECK(c1());
    CHECK(hipDeviceSynchronize());
    auto pab = snap(gab, ht * sizeof(float4)), pde = snap(gcd, ht * sizeof(float4)), pc = snap(ge, ht * sizeof(float2));
    CHECK(hipMemset(gab, 0, ht * sizeof(float4)));
    CHECK(hipMemset(gcd, 0, ht * sizeof(float4)));
    CHECK(hipMemset(ge, 0, ht * sizeof(float2)));
    auto c20 = [&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus, nullptr, 20); };
    CHECK(c20());
    CHECK(hipDeviceSynchronize());
    std::printf("cols half strips 2/CU vs production: gab, gde, gc\n");
    const bool same20 = (int)diff(snap(gab, ht * sizeof(float4)), pab) & (int)diff(snap(gcd, ht * sizeof(float4)), pde) &
                        (int)diff(snap(ge, ht * sizeof(float2)), pc);
    auto c22 = [&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus, nullptr, 22); };
    CHECK(hipMemset(gab, 0, ht * sizeof(float4)));
    CHECK(hipMemset(gcd, 0, ht * sizeof(float4)));
    CHECK(hipMemset(ge, 0, ht * sizeof(float2)));
    CHECK(c22());
    CHECK(hipDeviceSynchronize());
    std::printf("cols H in VGPRs (32 points per thread) vs production: gab, gde, gc\n");
    const bool same22 = (int)diff(snap(gab, ht * sizeof(float4)), pab) & (int)diff(snap(gcd, ht * sizeof(float4)), pde) &
                        (int)diff(snap(ge, ht * sizeof(float2)), pc);
    std::printf("H-in-VGPR fields bit-identical: %s\n", same22 ? "yes" : "NO");
    std::vector<std::vector<float>> tq(6);
    for (int r = 0; r < 7; r++)
    {
      tq[0].push_back(time_ms(c1, 10));
      tq[1].push_back(time_ms(c20, 10));
      tq[2].push_back(time_ms([&] { hipError_t e = c1(); return e == hipSuccess ? r1() : e; }, 10));
      tq[3].push_back(time_ms([&] { hipError_t e = c20(); return e == hipSuccess ? r1() : e; }, 10));
      tq[4].push_back(time_ms(c22, 10));
      tq[5].push_back(time_ms([&] { hipError_t e = c22(); return e == hipSuccess ? r1() : e; }, 10));
    }
    const char* qn[] = {"cols HS whole strips (production)", "cols HS half strips, 2/CU", "frame production",
                        "frame with half-strip cols", "cols H in VGPRs, 32 points/thread", "frame with H-in-VGPR cols"};
    for (int k = 0; k < 6; k++)
    {
      std::sort(tq[k].begin(), tq[k].end());
      std::printf("%-40s median %7.3f ms\n", qn[k], tq[k][3]);
    }
    std::printf("half-strip fields bit-identical: %s\n", same20 ? "yes" : "NO");
    if (quick)
      return 0;
  }
  {
    // persistent grids (resident blocks x CUs, item loop) against one-shot grids (one block per
    // item: launchers called with a huge CU count), same kernels, same results. The H-scratch
    // column pass needs one scratch slice per resident block, so its no-scratch forms stand in.
    const int BIG = 1 << 20;
    auto rp = [&] { return launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus); };
    auto ro = [&] { return launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, BIG); };
    auto wp = [&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, nullptr, 0, nullptr, 0); };
    auto wo = [&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, BIG, nullptr, 0, nullptr, 0); };
    auto hp = [&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, nullptr, 0, nullptr, 12); };
    auto ho = [&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, BIG, nullptr, 0, nullptr, 12); };
    const char* nm[] = {"rows persistent", "rows one-shot", "cols re-evolve persistent", "cols re-evolve one-shot",
                        "cols half2 persistent", "cols half2 one-shot"};
    std::vector<std::vector<float>> tt(6);
    for (int r = 0; r < 7; r++)
    {
      tt[0].push_back(time_ms(rp, 10));
      tt[1].push_back(time_ms(ro, 10));
      tt[2].push_back(time_ms(wp, 10));
      tt[3].push_back(time_ms(wo, 10));
      tt[4].push_back(time_ms(hp, 10));
      tt[5].push_back(time_ms(ho, 10));
    }
    for (int k = 0; k < 6; k++)
    {
      std::sort(tt[k].begin(), tt[k].end());
      std::printf("%-28s median %7.3f ms\n", nm[k], tt[k][3]);
    }
  }
  auto f00 = [&] { hipError_t e = c0(); return e == hipSuccess ? r0() : e; };
  auto f11 = [&] { hipError_t e = c1(); return e == hipSuccess ? r1() : e; };
  {
    // pass-1 cache-policy variants (HS): same results, timing only
    const char* vn[] = {"cols HS: production (nt h0 loads, nt stores)", "cols HS: default-policy h0 loads",
                        "cols HS: sc1 stores", "cols HS: sc1+nt stores"};
    std::vector<std::vector<float>> tv(4);
    for (int r = 0; r < 7; r++)
      for (int v = 0; v < 4; v++)
        tv[v].push_back(time_ms([&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus,
                                                                 nullptr, v); }, 10));
    for (int v = 0; v < 4; v++)
    {
      std::sort(tv[v].begin(), tv[v].end());
      std::printf("%-46s median %7.3f ms\n", vn[v], tv[v][3]);
    }
  }
  {
    // field layouts (row groups RG for gab/gde, RGC for gc; half_group_offset): pass 1 variant 7, 4, 6
    // with pass 2 variant 11, 8, 10. Only the intermediate layout changes, so the frame must be
    // bit-identical to the production frame.
    CHECK(f11());
    CHECK(hipDeviceSynchronize());
    auto pm = snap(maps, mb), pj = snap(jac, jb);
    const char* ln[] = {"production layout (RG 2, RGC 4)", "layout RG 1, RGC 1 (strips)", "layout RG 2, RGC 2",
                        "layout RG 4, RGC 4", "half strips RG 4, RGC 8 (cols2)", "half strips RG 2, RGC 4, dflt st",
                        "half strips RG 4, RGC 4, gc dflt st"};
    const int NV = 7, cv[] = {0, 7, 4, 6, 12, 13, 14}, rv[] = {0, 11, 8, 10, 12, 13, 14};
    bool same[7] = {true, true, true, true, true, true, true};
    for (int v = 1; v < NV; v++)
    {
      CHECK(hipMemset(maps, 0, mb));
      CHECK(hipMemset(jac, 0, jb));
      CHECK(launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus, nullptr, cv[v]));
      CHECK(launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus, rv[v]));
      CHECK(hipDeviceSynchronize());
      std::printf("%s vs production frame:\n", ln[v]);
      same[v] = (int)diff(snap(maps, mb), pm) & (int)diff(snap(jac, jb), pj);
    }
    std::vector<std::vector<float>> tc(NV), tr(NV), tf(NV);
    for (int r = 0; r < 7; r++)
      for (int v = 0; v < NV; v++)
      {
        auto cl = [&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus, nullptr, cv[v]); };
        auto rl = [&] { return launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus, rv[v]); };
        tc[v].push_back(time_ms(cl, 10));
        tr[v].push_back(time_ms(rl, 10));
        tf[v].push_back(time_ms([&] { hipError_t e = cl(); return e == hipSuccess ? rl() : e; }, 10));
      }
    for (int v = 0; v < NV; v++)
    {
      std::sort(tc[v].begin(), tc[v].end());
      std::sort(tr[v].begin(), tr[v].end());
      std::sort(tf[v].begin(), tf[v].end());
      std::printf("%-34s cols %7.3f  rows %7.3f  frame %7.3f ms (median)  bit-identical %s\n", ln[v], tc[v][3], tr[v][3],
                  tf[v][3], same[v] ? "yes" : "NO");
    }
  }
  const int rounds = 7, reps = 10;
  std::vector<std::vector<float>> t(7);
  for (int r = 0; r < rounds; r++)
  {
    t[0].push_back(time_ms(c0, reps));
    t[1].push_back(time_ms(c1, reps));
    t[2].push_back(time_ms(r0, reps));
    t[3].push_back(time_ms(r1, reps));
    t[4].push_back(time_ms(f00, reps));
    t[5].push_back(time_ms(f11, reps));
    t[6].push_back(time_ms(r2, reps));
  }
  const double kept = (n / 2.0 + 4) / n;
  const double b1 = 56 * kept, b2 = 40 * kept + 36;
  const char* names[] = {"cols: re-evolve per round", "cols: H scratch (HS)", "rows: one image per item",
                         "rows: both images (production)", "frame: baseline", "frame: HS + both images", "rows: both images, streamed (nt) loads"};
  const double bpp[] = {b1, b1, b2, b2, b1 + b2, b1 + b2, b2};
  for (int k = 0; k < 7; k++)
  {
    std::sort(t[k].begin(), t[k].end());
    const double med = t[k][t[k].size() / 2];
    std::printf("%-30s median %7.3f ms  min %7.3f ms  %7.1f GB/s algorithmic (%.1f B/pt)  %.3e pts/s\n", names[k],
                med, t[k][0], bpp[k] * pts / med / 1e6, bpp[k], pts / med * 1e3);
  }
  return 0;
}
