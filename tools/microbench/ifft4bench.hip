// ifft4bench.hip — standalone EncodeIFFT at N = 8192 / 16384: the in-place passes (rows, then
// columns held one or two per workgroup: 16/32-B pieces) against rows + the four-step column
// transform through a work slab of wc columns (k_cols4_step1/2), timed interleaved; the two results
// are compared (relative max error per image; the factorisations differ, so not bit-identical).
// Usage: ifft4bench
#include "all_kernels.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
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
  CHECK(launch());
  CHECK(hipDeviceSynchronize());
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

static std::vector<float2> table(int logn)
{
  const int n = 1 << logn, lb = logn / 2, tb = 1 << lb, ta = 1 << (logn - lb);
  std::vector<float2> tab(tb + ta);
  for (int e = 0; e < tb; e++)
    tab[e] = make_float2((float)std::cos(2 * M_PI * e / n), (float)std::sin(2 * M_PI * e / n));
  for (int e = 0; e < ta; e++)
    tab[tb + e] = make_float2((float)std::cos(2 * M_PI * (double)e * tb / n), (float)std::sin(2 * M_PI * (double)e * tb / n));
  return tab;
}

__global__ void fill_img(float4* p, size_t n)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
  {
    unsigned h = (unsigned)i * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    const float a = ((float)(h & 0xffff) - 32768.0f) * (1.0f / 32768.0f);
    p[i] = make_float4(a, 0.5f * a, -0.25f * a, 0.125f * a);
  }
}

// "mall": 2 images of 16384^2 (the bench's EncodeIFFT leg), rows + four-step columns through work slabs
// of 256 .. 2048 columns with the slab's accesses non-temporal (production) or default-policy: a slab
// of <= 128 MiB may stay in the 256 MiB Infinity Cache between step 1's stores and step 2's loads.
static int mall_mode(int cus)
{
  constexpr int logn = 14, n = 1 << logn, imgs = 2;
  const size_t tex = (size_t)n * n * imgs;
  float4 *img, *work;
  CHECK(hipMalloc(&img, tex * 16));
  CHECK(hipMalloc(&work, ifft_fourstep_work_texels(logn, 2048) * 16));
  hipLaunchKernelGGL(fill_img, dim3(4096), dim3(256), 0, 0, img, tex);
  auto t1 = table(logn), t2 = table(logn - 4);
  float2 *tw, *tw2;
  CHECK(hipMalloc(&tw, t1.size() * 8));
  CHECK(hipMalloc(&tw2, t2.size() * 8));
  CHECK(hipMemcpy(tw, t1.data(), t1.size() * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(tw2, t2.data(), t2.size() * 8, hipMemcpyHostToDevice));
  std::vector<float4> base(tex);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(base.data(), img, tex * 16, hipMemcpyDeviceToHost));
  struct R { int wc; bool nt; std::vector<float> t; };
  std::vector<R> rs;
  for (int wc : {256, 512, 1024, 2048})
    for (bool nt : {true, false})
      rs.push_back({wc, nt, {}});
  // every variant must give the production result bit for bit (same arithmetic, only the policy / slab width)
  std::vector<float4> ref(tex), got(tex);
  for (size_t k = 0; k < rs.size(); k++)
  {
    CHECK(hipMemcpy(img, base.data(), tex * 16, hipMemcpyHostToDevice));
    CHECK(launch_ifft_fourstep_ab(logn, imgs, img, work, rs[k].wc, tw, tw2, 0, cus, rs[k].nt));
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(k == 0 ? ref.data() : got.data(), img, tex * 16, hipMemcpyDeviceToHost));
    if (k > 0)
      std::printf("wc %4d %s: %s\n", rs[k].wc, rs[k].nt ? "nt     " : "default",
                  std::memcmp(ref.data(), got.data(), tex * 16) == 0 ? "bit-identical to wc 256 nt" : "DIFFERS");
  }
  for (int r = 0; r < 5; r++)
    for (auto& v : rs)
      v.t.push_back(time_ms([&] { return launch_ifft_fourstep_ab(logn, imgs, img, work, v.wc, tw, tw2, 0, cus, v.nt); }, 3));
  for (auto& v : rs)
  {
    std::sort(v.t.begin(), v.t.end());
    std::printf("2 x 16384^2 EncodeIFFT, slab %4d columns, slab %s  median %7.3f ms  %7.1f GB/s at 64 B/texel\n", v.wc,
                v.nt ? "nt     " : "default", v.t[2], 64.0 * tex / v.t[2] / 1e6);
  }
  return 0;
}

// "ci": 2 images of 16384^2, step 2 on 16 columns per 1024-thread workgroup (launch_ifft_fourstep,
// production) against 8 per 512-thread workgroup (as k_gen4_step2), through a work slab of 2048 columns
// and a whole-image work image; all bit-identical (the same per-column arithmetic). Round 5
// (profiles/r05_ifft4bench_ci.log): 10.00 / 10.62 / 10.64 / 11.67 ms: neither is kept.
static int ci_mode(int cus)
{
  constexpr int logn = 14, n = 1 << logn, imgs = 2;
  const size_t tex = (size_t)n * n * imgs;
  float4 *img, *work;
  CHECK(hipMalloc(&img, tex * 16));
  CHECK(hipMalloc(&work, ifft_fourstep_work_texels(logn, n) * 16));
  hipLaunchKernelGGL(fill_img, dim3(4096), dim3(256), 0, 0, img, tex);
  auto t1 = table(logn), t2 = table(logn - 4);
  float2 *tw, *tw2;
  CHECK(hipMalloc(&tw, t1.size() * 8));
  CHECK(hipMalloc(&tw2, t2.size() * 8));
  CHECK(hipMemcpy(tw, t1.data(), t1.size() * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(tw2, t2.data(), t2.size() * 8, hipMemcpyHostToDevice));
  std::vector<float4> base(tex), ref(tex), got(tex);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(base.data(), img, tex * 16, hipMemcpyDeviceToHost));
  struct R { const char* name; int wc; int ci8; std::vector<float> t; };
  std::vector<R> rs = {{"CI 16, slab 2048", 2048, 0, {}}, {"CI 8, slab 2048", 2048, 1, {}},
                       {"CI 16, whole image", n, 0, {}}, {"CI 8, whole image", n, 1, {}},
                       {"CI 8 MINB 4, slab 2048", 2048, 2, {}}, {"CI 8 MINB 4, slab 4096", 4096, 2, {}},
                       {"CI 8 MINB 4 PF 4 res, slab 2048", 2048, 3, {}}, {"CI 8 MINB 4, whole image", n, 2, {}}};
  // CI 8: rows, then per image and slab step 1 + k_cols4_step2<10, true, 8> (512-thread workgroups);
  // variant 2: k_cols4_step2e<10, 0, 8, 4> (<= 128 VGPRs, two workgroups per CU), 3: PF 4 on a resident grid
  auto ci8 = [&](int wc, int var) -> hipError_t {
    hipError_t e = launch_rows_ifft(logn, imgs, img, tw, 0, cus);
    if (e != hipSuccess)
      return e;
    using S2 = FftShape<logn - 4>;
    constexpr int CI = 8, WG2 = S2::T * CI;
    auto k1 = k_cols4_step1<logn>;
    auto k2 = k_cols4_step2<logn - 4, true, CI>;
    const int lds2 = ((S2::TW_ENTRIES * 8 + 15) / 16) * 16 + CI * S2::PADDED * 8;
    for (int im = 0; im < imgs; im++)
      for (int x0 = 0; x0 < n; x0 += wc)
      {
        float4* im0 = img + ((size_t)im << (2 * logn));
        const int g1 = persistent_grid(k1, 256, 0, (wc / 64) * ((n / 16) / 4), cus);
        hipLaunchKernelGGL(k1, dim3(g1), dim3(256), 0, 0, 1, x0, wc, im0, work, tw);
        if (var == 1)
        {
          const int g2 = persistent_grid(k2, WG2, lds2, 16 * (wc / CI), cus);
          hipLaunchKernelGGL(k2, dim3(g2), dim3(WG2), lds2, 0, 1, x0, wc, work, im0, tw2);
        }
        else if (var == 2)
        {
          auto k2m = k_cols4_step2e<logn - 4, 0, CI, 4>;
          const int g2 = persistent_grid(k2m, WG2, lds2, 16 * (wc / CI), cus);
          hipLaunchKernelGGL(k2m, dim3(g2), dim3(WG2), lds2, 0, 1, x0, wc, work, im0, tw2);
        }
        else
        {
          auto k2m = k_cols4_step2e<logn - 4, 4, CI, 4>;
          const int g2 = resident_grid(k2m, WG2, lds2, 16 * (wc / CI), cus);
          hipLaunchKernelGGL(k2m, dim3(g2), dim3(WG2), lds2, 0, 1, x0, wc, work, im0, tw2);
        }
      }
    return hipGetLastError();
  };
  auto run = [&](const R& v) {
    return v.ci8 ? ci8(v.wc, v.ci8) : launch_ifft_fourstep(logn, imgs, img, work, v.wc, tw, tw2, 0, cus);
  };
  for (size_t k = 0; k < rs.size(); k++)
  {
    CHECK(hipMemcpy(img, base.data(), tex * 16, hipMemcpyHostToDevice));
    CHECK(run(rs[k]));
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(k == 0 ? ref.data() : got.data(), img, tex * 16, hipMemcpyDeviceToHost));
    if (k > 0)
      std::printf("%s: %s\n", rs[k].name, std::memcmp(ref.data(), got.data(), tex * 16) == 0 ? "bit-identical" : "DIFFERS");
  }
  for (int r = 0; r < 5; r++)
    for (auto& v : rs)
      v.t.push_back(time_ms([&] { return run(v); }, 3));
  for (auto& v : rs)
  {
    std::sort(v.t.begin(), v.t.end());
    std::printf("2 x 16384^2 EncodeIFFT, %-20s median %7.3f ms\n", v.name, v.t[2]);
  }
  return 0;
}

// "early": 2 images of 16384^2 through a 2048-column work slab; step 2 as production (one-shot grid)
// against k_cols4_step2e (resident grid, the next item's first PF loads before this item's stores),
// PF = 0 / 4 / 8 / 16; all bit-identical (round 6).
static int early_mode(int cus)
{
  constexpr int logn = 14, n = 1 << logn, imgs = 2, wc = 2048;
  const size_t tex = (size_t)n * n * imgs;
  float4 *img, *work;
  CHECK(hipMalloc(&img, tex * 16));
  CHECK(hipMalloc(&work, ifft_fourstep_work_texels(logn, wc) * 16));
  hipLaunchKernelGGL(fill_img, dim3(4096), dim3(256), 0, 0, img, tex);
  auto t1 = table(logn), t2 = table(logn - 4);
  float2 *tw, *tw2;
  CHECK(hipMalloc(&tw, t1.size() * 8));
  CHECK(hipMalloc(&tw2, t2.size() * 8));
  CHECK(hipMemcpy(tw, t1.data(), t1.size() * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(tw2, t2.data(), t2.size() * 8, hipMemcpyHostToDevice));
  std::vector<float4> base(tex), ref(tex), got(tex);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(base.data(), img, tex * 16, hipMemcpyDeviceToHost));
  using S2 = FftShape<logn - 4>;
  using K2 = ColCfg<logn - 4>;
  const int lds2 = lds_bytes_cols<logn - 4>();
  auto with_step2 = [&](auto k2, bool resident, bool blocked = false) {
    return std::function<hipError_t()>([=] {
      hipError_t e = launch_rows_ifft(logn, imgs, img, tw, 0, cus);
      if (e != hipSuccess)
        return e;
      auto k1 = blocked ? k_cols4_step1b<logn> : k_cols4_step1<logn>;
      for (int im = 0; im < imgs; im++)
        for (int x0 = 0; x0 < n; x0 += wc)
        {
          float4* im0 = img + ((size_t)im << (2 * logn));
          const int g1 = persistent_grid(k1, 256, 0, (wc / 64) * ((n / 16) / 4), cus);
          hipLaunchKernelGGL(k1, dim3(g1), dim3(256), 0, 0, 1, x0, wc, im0, work, tw);
          const int items = 16 * (wc / K2::C);
          const int g2 = resident ? resident_grid(k2, K2::WG, lds2, items, cus) : persistent_grid(k2, K2::WG, lds2, items, cus);
          hipLaunchKernelGGL(k2, dim3(g2), dim3(K2::WG), lds2, 0, 1, x0, wc, work, im0, tw2);
        }
      return hipGetLastError();
    });
  };
  std::vector<std::string> names = {"production (one-shot)", "step2e PF 0 (resident)", "step2e PF 4", "step2e PF 8",
                                    "step2e PF 16", "step2e PF 0 one-shot"};
  std::vector<std::function<hipError_t()>> runs = {
      with_step2(k_cols4_step2<logn - 4>, false), with_step2(k_cols4_step2e<logn - 4, 0>, true),
      with_step2(k_cols4_step2e<logn - 4, 4>, true), with_step2(k_cols4_step2e<logn - 4, 8>, true),
      with_step2(k_cols4_step2e<logn - 4, 16>, true), with_step2(k_cols4_step2e<logn - 4, 0>, false)};
  names.push_back("slab blocked in 16-column strips");
  runs.push_back(with_step2(k_cols4_step2b<logn - 4>, false, true));
  // the row pass alone: production k_rows_ifft (one-shot) against k_rows_ifft_early PF 0 / 4 / 8 (resident)
  const int ldsr = lds_bytes_rows<logn>();
  auto rows_with = [&](auto kern, bool resident) {
    return std::function<hipError_t()>([=] {
      const int items = imgs * n;
      const int g = resident ? resident_grid(kern, RowCfg<logn>::WG, ldsr, items, cus)
                             : persistent_grid(kern, RowCfg<logn>::WG, ldsr, items, cus);
      hipLaunchKernelGGL(kern, dim3(g), dim3(RowCfg<logn>::WG), ldsr, 0, items, img, tw);
      return hipGetLastError();
    });
  };
  const size_t first_rows = runs.size();
  names.insert(names.end(), {"rows: production (one-shot)", "rows: early PF 0 (resident)", "rows: early PF 4",
                             "rows: early PF 8"});
  runs.insert(runs.end(), {rows_with(k_rows_ifft<logn>, false), rows_with(k_rows_ifft_early<logn, 0>, true),
                           rows_with(k_rows_ifft_early<logn, 4>, true), rows_with(k_rows_ifft_early<logn, 8>, true)});
  (void)sizeof(S2);
  for (size_t k = 0; k < runs.size(); k++)
  {
    const bool first = k == 0 || k == first_rows;
    CHECK(hipMemcpy(img, base.data(), tex * 16, hipMemcpyHostToDevice));
    CHECK(runs[k]());
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(first ? ref.data() : got.data(), img, tex * 16, hipMemcpyDeviceToHost));
    if (!first)
      std::printf("%s: %s\n", names[k].c_str(), std::memcmp(ref.data(), got.data(), tex * 16) == 0 ? "bit-identical" : "DIFFERS");
  }
  std::vector<std::vector<float>> t(runs.size());
  for (int r = 0; r < 5; r++)
    for (size_t k = 0; k < runs.size(); k++)
      t[k].push_back(time_ms(runs[k], 3));
  for (size_t k = 0; k < runs.size(); k++)
  {
    std::sort(t[k].begin(), t[k].end());
    std::printf("2 x 16384^2 EncodeIFFT, %-30s median %7.3f ms\n", names[k].c_str(), t[k][2]);
  }
  return 0;
}


// "occ" (round 6): 2 images of 16384^2 through a 2048-column slab; step 1 at 138 VGPRs (three 256-thread
// workgroups per CU; MINW 1) or <= 128 (four; MINW 4, 28 B of spills) against step 2 on 16 columns per
// 1024-thread workgroup or 8 per 512-thread workgroup at <= 128 VGPRs (two per CU). Each combination is
// timed whole (rows + columns) and per step (the slabs' step-1 or step-2 launches alone).
static int occ_mode(int cus)
{
  constexpr int logn = 14, n = 1 << logn, imgs = 2, wc = 2048;
  const size_t tex = (size_t)n * n * imgs;
  float4 *img, *work;
  CHECK(hipMalloc(&img, tex * 16));
  CHECK(hipMalloc(&work, ifft_fourstep_work_texels(logn, wc) * 16));
  hipLaunchKernelGGL(fill_img, dim3(4096), dim3(256), 0, 0, img, tex);
  auto t1 = table(logn), t2 = table(logn - 4);
  float2 *tw, *tw2;
  CHECK(hipMalloc(&tw, t1.size() * 8));
  CHECK(hipMalloc(&tw2, t2.size() * 8));
  CHECK(hipMemcpy(tw, t1.data(), t1.size() * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(tw2, t2.data(), t2.size() * 8, hipMemcpyHostToDevice));
  std::vector<float4> base(tex), ref(tex), got(tex);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(base.data(), img, tex * 16, hipMemcpyDeviceToHost));
  using S2 = FftShape<logn - 4>;
  // parts: 1 = rows, 2 = step 1, 4 = step 2
  auto make = [&](auto k1, auto k2, int ci, int parts) {
    return std::function<hipError_t()>([=] {
      if (parts & 1)
      {
        hipError_t e = launch_rows_ifft(logn, imgs, img, tw, 0, cus);
        if (e != hipSuccess)
          return e;
      }
      const int wg2 = S2::T * ci, lds2 = ((S2::TW_ENTRIES * 8 + 15) / 16) * 16 + ci * S2::PADDED * 8;
      for (int im = 0; im < imgs; im++)
        for (int x0 = 0; x0 < n; x0 += wc)
        {
          float4* im0 = img + ((size_t)im << (2 * logn));
          if (parts & 2)
          {
            const int g1 = persistent_grid(k1, 256, 0, (wc / 64) * ((n / 16) / 4), cus);
            hipLaunchKernelGGL(k1, dim3(g1), dim3(256), 0, 0, 1, x0, wc, im0, work, tw);
          }
          if (parts & 4)
          {
            const int g2 = persistent_grid(k2, wg2, lds2, 16 * (wc / ci), cus);
            hipLaunchKernelGGL(k2, dim3(g2), dim3(wg2), lds2, 0, 1, x0, wc, work, im0, tw2);
          }
        }
      return hipGetLastError();
    });
  };
  auto s1a = k_cols4_step1<logn, true, 1>;
  auto s1b = k_cols4_step1<logn, true, 4>;
  auto s2a = k_cols4_step2<logn - 4, true, 16>;
  auto s2b = k_cols4_step2<logn - 4, true, 8>;
  std::vector<std::string> names = {"step1 MINW 1 + step2 CI 16 (r06e production)", "step1 MINW 4 + step2 CI 16",
                                    "step1 MINW 1 + step2 CI 8 MINW 4", "step1 MINW 4 + step2 CI 8 MINW 4",
                                    "step 1 alone, MINW 1", "step 1 alone, MINW 4", "step 2 alone, CI 16",
                                    "step 2 alone, CI 8 MINW 4"};
  std::vector<std::function<hipError_t()>> runs = {make(s1a, s2a, 16, 7), make(s1b, s2a, 16, 7), make(s1a, s2b, 8, 7),
                                                   make(s1b, s2b, 8, 7), make(s1a, s2a, 16, 2), make(s1b, s2a, 16, 2),
                                                   make(s1a, s2a, 16, 4), make(s1a, s2b, 8, 4)};
  for (size_t k = 0; k < 4; k++)
  {
    CHECK(hipMemcpy(img, base.data(), tex * 16, hipMemcpyHostToDevice));
    CHECK(runs[k]());
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(k == 0 ? ref.data() : got.data(), img, tex * 16, hipMemcpyDeviceToHost));
    if (k > 0)
      std::printf("%s: %s\n", names[k].c_str(), std::memcmp(ref.data(), got.data(), tex * 16) == 0 ? "bit-identical" : "DIFFERS");
  }
  std::vector<std::vector<float>> t(runs.size());
  for (int r = 0; r < 7; r++)
    for (size_t k = 0; k < runs.size(); k++)
      t[k].push_back(time_ms(runs[k], 3));
  for (size_t k = 0; k < runs.size(); k++)
  {
    std::sort(t[k].begin(), t[k].end());
    std::printf("2 x 16384^2 EncodeIFFT, %-46s median %7.3f ms (min %7.3f)\n", names[k].c_str(), t[k][3], t[k][0]);
  }
  return 0;
}

// "pipe" (round 6): 2 images of 16384^2; the column steps of consecutive slabs overlapped on two streams
// with two work slabs: step 1 of slab s + 1 (streaming, 256-thread workgroups) beside step 2 of slab s
// (LDS-bound, 1024-thread workgroups), against production (one stream). Bit-identical by construction.
static int pipe_mode(int cus)
{
  constexpr int logn = 14, n = 1 << logn, imgs = 2;
  const size_t tex = (size_t)n * n * imgs;
  float4 *img, *work;
  CHECK(hipMalloc(&img, tex * 16));
  CHECK(hipMalloc(&work, 2 * ifft_fourstep_work_texels(logn, 4096) * 16));
  hipLaunchKernelGGL(fill_img, dim3(4096), dim3(256), 0, 0, img, tex);
  auto t1 = table(logn), t2 = table(logn - 4);
  float2 *tw, *tw2;
  CHECK(hipMalloc(&tw, t1.size() * 8));
  CHECK(hipMalloc(&tw2, t2.size() * 8));
  CHECK(hipMemcpy(tw, t1.data(), t1.size() * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(tw2, t2.data(), t2.size() * 8, hipMemcpyHostToDevice));
  std::vector<float4> base(tex), ref(tex), got(tex);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(base.data(), img, tex * 16, hipMemcpyDeviceToHost));
  hipStream_t sb;
  CHECK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  constexpr int kMaxSlabs = 64;
  hipEvent_t e1[kMaxSlabs], e2[kMaxSlabs], er;
  for (int k = 0; k < kMaxSlabs; k++)
  {
    CHECK(hipEventCreateWithFlags(&e1[k], hipEventDisableTiming));
    CHECK(hipEventCreateWithFlags(&e2[k], hipEventDisableTiming));
  }
  CHECK(hipEventCreateWithFlags(&er, hipEventDisableTiming));
  using K2 = ColCfg<logn - 4>;
  const int lds2 = lds_bytes_cols<logn - 4>();
  auto k1 = k_cols4_step1<logn>;
  auto k2 = k_cols4_step2<logn - 4>;
  auto piped = [&](int wc, int cap1, int cap2) {
    return std::function<hipError_t()>([=] {
      hipError_t e = launch_rows_ifft(logn, imgs, img, tw, 0, cus);
      if (e != hipSuccess)
        return e;
      const size_t wslab = ifft_fourstep_work_texels(logn, wc);
      int s = 0;
      for (int im = 0; im < imgs; im++)
        for (int x0 = 0; x0 < n; x0 += wc, s++)
        {
          float4* im0 = img + ((size_t)im << (2 * logn));
          float4* w = work + (s & 1) * wslab;
          if (s >= 2)
            CHECK(hipStreamWaitEvent(0, e2[s - 2], 0));  // slab s - 2's step 2 has read this work slab
          const int g1 = std::min(cap1, persistent_grid(k1, 256, 0, (wc / 64) * ((n / 16) / 4), cus));
          hipLaunchKernelGGL(k1, dim3(g1), dim3(256), 0, 0, 1, x0, wc, im0, w, tw);
          CHECK(hipEventRecord(e1[s], 0));
          CHECK(hipStreamWaitEvent(sb, e1[s], 0));
          const int g2 = std::min(cap2, persistent_grid(k2, K2::WG, lds2, 16 * (wc / K2::C), cus));
          hipLaunchKernelGGL(k2, dim3(g2), dim3(K2::WG), lds2, sb, 1, x0, wc, w, im0, tw2);
          CHECK(hipEventRecord(e2[s], sb));
        }
      CHECK(hipEventRecord(er, sb));
      CHECK(hipStreamWaitEvent(0, er, 0));
      return hipGetLastError();
    });
  };
  std::vector<std::string> names = {"production (one stream, slab 2048)", "piped, slab 2048", "piped, slab 1024",
                                    "piped, slab 4096", "piped, slab 2048, step 2 on 192 CUs' grid",
                                    "piped, slab 2048, step 1 grid 256"};
  std::vector<std::function<hipError_t()>> runs = {
      std::function<hipError_t()>([=] { return launch_ifft_fourstep(logn, imgs, img, work, 2048, tw, tw2, 0, cus); }),
      piped(2048, 1 << 30, 1 << 30), piped(1024, 1 << 30, 1 << 30), piped(4096, 1 << 30, 1 << 30),
      piped(2048, 1 << 30, 192), piped(2048, 256, 1 << 30)};
  for (size_t k = 0; k < runs.size(); k++)
  {
    CHECK(hipMemcpy(img, base.data(), tex * 16, hipMemcpyHostToDevice));
    CHECK(runs[k]());
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(k == 0 ? ref.data() : got.data(), img, tex * 16, hipMemcpyDeviceToHost));
    if (k > 0)
      std::printf("%s: %s\n", names[k].c_str(), std::memcmp(ref.data(), got.data(), tex * 16) == 0 ? "bit-identical" : "DIFFERS");
  }
  std::vector<std::vector<float>> t(runs.size());
  for (int r = 0; r < 7; r++)
    for (size_t k = 0; k < runs.size(); k++)
      t[k].push_back(time_ms(runs[k], 3));
  for (size_t k = 0; k < runs.size(); k++)
  {
    std::sort(t[k].begin(), t[k].end());
    std::printf("2 x 16384^2 EncodeIFFT, %-46s median %7.3f ms (min %7.3f)\n", names[k].c_str(), t[k][3], t[k][0]);
  }
  return 0;
}

int main(int argc, char** argv)
{
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  if (argc > 1 && std::strcmp(argv[1], "mall") == 0)
    return mall_mode(cus);
  if (argc > 1 && std::strcmp(argv[1], "ci") == 0)
    return ci_mode(cus);
  if (argc > 1 && std::strcmp(argv[1], "pipe") == 0)
    return pipe_mode(cus);
  if (argc > 1 && std::strcmp(argv[1], "occ") == 0)
    return occ_mode(cus);
  if (argc > 1 && std::strcmp(argv[1], "early") == 0)
    return early_mode(cus);
  for (int logn : {13, 14})
  {
    const int n = 1 << logn, imgs = logn == 13 ? (argc > 1 ? std::atoi(argv[1]) : 4) : 1;
    const size_t tex = (size_t)n * n * imgs;
    std::vector<float4> h(tex);
    uint32_t st = 12345;
    for (size_t k = 0; k < tex; k++)
    {
      st = st * 1664525u + 1013904223u;
      const float a = (st >> 8) * (1.0f / 16777216.0f) - 0.5f;
      h[k] = make_float4(a, 0.5f * a, std::sin(0.001f * (float)(k % 9973)), -0.25f * a);
    }
    float4 *img, *ref, *work;
    CHECK(hipMalloc(&img, tex * 16));
    CHECK(hipMalloc(&ref, tex * 16));
    CHECK(hipMalloc(&work, std::max(ifft_fourstep_work_texels(logn, n), tex) * 16));
    auto t1 = table(logn), t2 = table(logn - 4);
    float2 *tw, *tw2;
    CHECK(hipMalloc(&tw, t1.size() * 8));
    CHECK(hipMalloc(&tw2, t2.size() * 8));
    CHECK(hipMemcpy(tw, t1.data(), t1.size() * 8, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(tw2, t2.data(), t2.size() * 8, hipMemcpyHostToDevice));
    // reference: in-place rows + columns
    CHECK(hipMemcpy(ref, h.data(), tex * 16, hipMemcpyHostToDevice));
    CHECK(launch_rows_ifft(logn, imgs, ref, tw, 0, cus));
    CHECK(launch_cols(logn, imgs, ref, tw, 0, cus));
    CHECK(hipDeviceSynchronize());
    std::vector<float4> a(tex), b(tex);
    CHECK(hipMemcpy(a.data(), ref, tex * 16, hipMemcpyDeviceToHost));
    const int wcs[] = {512, 1024, 2048, n};
    for (int wc : wcs)
    {
      CHECK(hipMemcpy(img, h.data(), tex * 16, hipMemcpyHostToDevice));
      CHECK(launch_ifft_fourstep(logn, imgs, img, work, wc, tw, tw2, 0, cus));
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemcpy(b.data(), img, tex * 16, hipMemcpyDeviceToHost));
      double mx = 0, er = 0;
      for (size_t k = 0; k < tex; k++)
      {
        const float* x = &a[k].x;
        const float* y = &b[k].x;
        for (int j = 0; j < 4; j++)
        {
          mx = std::max(mx, (double)std::fabs(x[j]));
          er = std::max(er, (double)std::fabs(x[j] - y[j]));
        }
      }
      std::printf("N=%d wc=%d: four-step vs in-place max |diff| / max |x| = %.3g\n", n, wc, er / mx);
    }
    std::vector<std::string> names = {"in place rows + cols"};
    std::vector<std::function<hipError_t()>> runs = {[&] {
      hipError_t e = launch_rows_ifft(logn, imgs, img, tw, 0, cus);
      return e == hipSuccess ? launch_cols(logn, imgs, img, tw, 0, cus) : e;
    }};
    for (int wc : wcs)
    {
      names.push_back("rows + four-step cols, wc " + std::to_string(wc));
      runs.push_back([&, wc] { return launch_ifft_fourstep(logn, imgs, img, work, wc, tw, tw2, 0, cus); });
    }
    // in-place columns with more strips per XCD group (their partial lines meet in one L2)
    names.push_back("in place rows + cols, 4 strips per XCD group");
    runs.push_back([&] {
      hipError_t e = launch_rows_ifft(logn, imgs, img, tw, 0, cus);
      return e == hipSuccess ? launch_cols_group<4>(logn, imgs, img, tw, 0, cus) : e;
    });
    names.push_back("in place rows + cols, 8 strips per XCD group");
    runs.push_back([&] {
      hipError_t e = launch_rows_ifft(logn, imgs, img, tw, 0, cus);
      return e == hipSuccess ? launch_cols_group<8>(logn, imgs, img, tw, 0, cus) : e;
    });
    names.push_back("cols only in place (production group)");
    runs.push_back([&] { return launch_cols(logn, imgs, img, tw, 0, cus); });
    names.push_back("cols only, 4 strips per XCD group");
    runs.push_back([&] { return launch_cols_group<4>(logn, imgs, img, tw, 0, cus); });
    names.push_back("cols only, 8 strips per XCD group");
    runs.push_back([&] { return launch_cols_group<8>(logn, imgs, img, tw, 0, cus); });
    if (logn == 13)
    {
      // column-first through a work image (the strided pass only reads 32-B pieces, which L2
      // merges; it writes whole strips), then the blocked row pass, whose 128-B lines hold 4 rows =
      // 2 items: GRPR items per XCD group read them together
      for (int grpr : {1, 2, 4})
      {
        CHECK(hipMemcpy(img, h.data(), tex * 16, hipMemcpyHostToDevice));
        hipError_t ec = grpr == 1 ? launch_ifft_colfirst13<2, 1>(imgs, img, work, tw, 0, cus)
                        : grpr == 2 ? launch_ifft_colfirst13<2, 2>(imgs, img, work, tw, 0, cus)
                                    : launch_ifft_colfirst13<2, 4>(imgs, img, work, tw, 0, cus);
        CHECK(ec);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(b.data(), img, tex * 16, hipMemcpyDeviceToHost));
        double mx = 0, er = 0;
        for (size_t k = 0; k < tex; k++)
          for (int j = 0; j < 4; j++)
          {
            mx = std::max(mx, (double)std::fabs((&a[k].x)[j]));
            er = std::max(er, (double)std::fabs((&a[k].x)[j] - (&b[k].x)[j]));
          }
        std::printf("N=%d column-first, row items grouped %d: vs in-place max |diff| / max |x| = %.3g\n", n, grpr,
                    er / mx);
        names.push_back("column-first via work image, row items grouped " + std::to_string(grpr));
        runs.push_back([&, grpr] {
          return grpr == 1 ? launch_ifft_colfirst13<2, 1>(imgs, img, work, tw, 0, cus)
                           : grpr == 2 ? launch_ifft_colfirst13<2, 2>(imgs, img, work, tw, 0, cus)
                                       : launch_ifft_colfirst13<2, 4>(imgs, img, work, tw, 0, cus);
        });
      }
      // one row per row-pass item (512 threads, half the LDS: two workgroups per CU), the 4 items of a
      // line grouped on one XCD (4) or 8 items (two lines of a strip piece)
      for (int grpr : {4, 8})
      {
        auto run = [&, grpr] {
          return grpr == 4 ? launch_ifft_colfirst_ab<13, 2, 4, 1>(imgs, img, work, tw, 0, cus)
                           : launch_ifft_colfirst_ab<13, 2, 8, 1>(imgs, img, work, tw, 0, cus);
        };
        CHECK(hipMemcpy(img, h.data(), tex * 16, hipMemcpyHostToDevice));
        CHECK(run());
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(b.data(), img, tex * 16, hipMemcpyDeviceToHost));
        double mx = 0, er = 0;
        for (size_t k = 0; k < tex; k++)
          for (int j = 0; j < 4; j++)
          {
            mx = std::max(mx, (double)std::fabs((&a[k].x)[j]));
            er = std::max(er, (double)std::fabs((&a[k].x)[j] - (&b[k].x)[j]));
          }
        std::printf("N=%d column-first, one-row items grouped %d: vs in-place max |diff| / max |x| = %.3g\n", n, grpr,
                    er / mx);
        names.push_back("column-first, one-row items grouped " + std::to_string(grpr));
        runs.push_back(run);
      }
    }
    if (logn == 14)
    {
      // column-first through a work image at 16384 (one-column strided items: 16-B read pieces,
      // 8 strips per line; whole strips written), blocked rows with 8 row items per XCD group
      CHECK(hipFree(work));
      CHECK(hipMalloc(&work, tex * 16));
      for (int v = 0; v < 3; v++)
      {
        auto run = [&, v] {
          return v == 0 ? launch_ifft_colfirst_ab<14, 8, 8>(imgs, img, work, tw, 0, cus)
                 : v == 1 ? launch_ifft_colfirst_ab<14, 8, 1>(imgs, img, work, tw, 0, cus)
                          : launch_ifft_colfirst_ab<14, 2, 8>(imgs, img, work, tw, 0, cus);
        };
        CHECK(hipMemcpy(img, h.data(), tex * 16, hipMemcpyHostToDevice));
        CHECK(run());
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(b.data(), img, tex * 16, hipMemcpyDeviceToHost));
        double mx = 0, er = 0;
        for (size_t k = 0; k < tex; k++)
          for (int j = 0; j < 4; j++)
          {
            mx = std::max(mx, (double)std::fabs((&a[k].x)[j]));
            er = std::max(er, (double)std::fabs((&a[k].x)[j] - (&b[k].x)[j]));
          }
        const char* nm[3] = {"column-first, col group 8, row group 8", "column-first, col group 8, rows ungrouped",
                             "column-first, col group 2, row group 8"};
        std::printf("N=%d %s: vs in-place max |diff| / max |x| = %.3g\n", n, nm[v], er / mx);
        names.push_back(nm[v]);
        runs.push_back(run);
      }
    }
    std::vector<std::vector<float>> t(runs.size());
    for (int r = 0; r < 5; r++)
      for (size_t k = 0; k < runs.size(); k++)
        t[k].push_back(time_ms(runs[k], 3));
    for (size_t k = 0; k < runs.size(); k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::printf("N=%d x%d %-36s median %7.3f ms\n", n, imgs, names[k].c_str(), t[k][2]);
    }
    CHECK(hipFree(img));
    CHECK(hipFree(ref));
    CHECK(hipFree(work));
    CHECK(hipFree(tw));
    CHECK(hipFree(tw2));
  }
  return 0;
}
