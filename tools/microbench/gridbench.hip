// gridbench.hip — persistent grids (resident blocks x CUs, item loop) against one-shot grids (one
// block per work item, the hardware dispatcher hands out items) for the production frame and
// EncodeIFFT kernels, timed interleaved in one process. The launchers' default is the one-shot grid
// (all CUs available); g_force_persistent gives the persistent grid of the same kernel.
// Also times the in-place EncodeIFFT passes at 8192 and 16384 (rows then columns).
// Usage: gridbench
#include "all_kernels.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
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

// persistent grid through the production launchers (their default is one-shot with all CUs)
template <typename F>
static hipError_t persist(F&& f)
{
  g_force_persistent = true;
  const hipError_t e = f();
  g_force_persistent = false;
  return e;
}

static float2* make_twiddles(int logn)
{
  const int n = 1 << logn, lb = logn / 2, tb = 1 << lb, ta = 1 << (logn - lb);
  std::vector<float2> tab(tb + ta);
  for (int e = 0; e < tb; e++)
    tab[e] = make_float2((float)std::cos(2 * M_PI * e / n), (float)std::sin(2 * M_PI * e / n));
  for (int e = 0; e < ta; e++)
    tab[tb + e] = make_float2((float)std::cos(2 * M_PI * e * tb / n), (float)std::sin(2 * M_PI * e * tb / n));
  float2* tw;
  CHECK(hipMalloc(&tw, tab.size() * sizeof(float2)));
  CHECK(hipMemcpy(tw, tab.data(), tab.size() * sizeof(float2), hipMemcpyHostToDevice));
  return tw;
}

struct Case
{
  std::string name;
  double bytes;  // algorithmic bytes per call
  std::function<hipError_t()> run;
  std::vector<float> t;
};

static void run_cases(std::vector<Case>& cs, int rounds, int reps)
{
  for (int r = 0; r < rounds; r++)
    for (auto& c : cs)
      c.t.push_back(time_ms(c.run, reps));
  for (auto& c : cs)
  {
    std::sort(c.t.begin(), c.t.end());
    const float med = c.t[c.t.size() / 2];
    std::printf("%-52s median %7.3f ms  %7.1f GB/s\n", c.name.c_str(), med, c.bytes / med / 1e6);
  }
}

int main()
{
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int BIG = 1 << 20;
  {
    // generator frame at 8 x 4096^2 (half spectrum)
    const int logn = 12, n = 1 << logn, C = 8;
    const size_t tex = (size_t)n * n;
    float4 *h0, *maps, *gab, *gcd, *spec;
    float2 *ge, *hs;
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
    float2* tw = make_twiddles(logn);
    FrameParams fp{};
    FoamParams foam{};
    fp.cascades = C;
    static const float planes[] = {5, 17, 101, 251, 509, 1021, 2039, 4093};
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
      s.planeSize = planes[c];
      s.scale = 1;
      s.spread = 0.2f;
      CHECK(launch_generate_spectrum(s, n, h0 + tex * c, 0, cus));
      fp.c[c] = {2.0f * 3.14159265358f / s.planeSize, 37.5f, s.g, s.h};
      foam.displacement[c] = s.displacement;
    }
    CHECK(launch_half_columns(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus));
    CHECK(hipDeviceSynchronize());
    const double pts = (double)tex * C, kept = (n / 2.0 + 4) / n;
    std::vector<Case> cs = {
        {"4096 cols HS (production, persistent)", 56 * kept * pts,
         [&] { return launch_half_columns(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus); }},
        {"4096 rows persistent (round-1 default)", (40 * kept + 36) * pts,
         [&] { return persist([&] { return launch_half_rows(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus); }); }},
        {"4096 rows one-shot", (40 * kept + 36) * pts,
         [&] { return launch_half_rows(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, BIG); }},
    };
    run_cases(cs, 7, 10);
    CHECK(hipFree(h0));
    CHECK(hipFree(jac));
    CHECK(hipFree(gab));
    CHECK(hipFree(gcd));
    CHECK(hipFree(ge));
    CHECK(hipFree(spec));
    CHECK(hipFree(hs));
    CHECK(hipFree(tw));
    // EncodeIFFT at 4096: 8 images through the work image (maps reused as the images)
    float4* work;
    CHECK(hipMalloc(&work, tex * 8 * sizeof(float4)));
    float2* tw12 = make_twiddles(12);
    using K = ColFirstCfg<12>;
    using S = FftShape<12>;
    const int twb = ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
    auto rows2 = k_rows_final<12, true, kStream, kStream, 2>;
    const int lds2 = twb + lds_row_slots<12>(2) * 8;
    CHECK(hipFuncSetAttribute((const void*)rows2, hipFuncAttributeMaxDynamicSharedMemorySize, lds2));
    auto cols = k_cols_to_blocks<12>;
    const int lds1 = twb + K::LDS1;
    CHECK(hipFuncSetAttribute((const void*)cols, hipFuncAttributeMaxDynamicSharedMemorySize, lds1));
    auto rows4 = k_rows_final<12, true>;
    CHECK(hipFuncSetAttribute((const void*)rows4, hipFuncAttributeMaxDynamicSharedMemorySize, twb + K::LDS2));
    const SlabGeom g{0, n};
    const double ib = 32.0 * tex * 8;
    std::vector<Case> ci = {
        {"ifft4096 x8 both passes persistent (round-1 default)", 2 * ib,
         [&] { return persist([&] { return launch_ifft_colfirst(12, 8, maps, work, tw12, 0, cus); }); }},
        {"ifft4096 x8 both passes one-shot", 2 * ib, [&] { return launch_ifft_colfirst(12, 8, maps, work, tw12, 0, BIG); }},
        {"ifft4096 cols_to_blocks persistent", ib,
         [&] {
           hipLaunchKernelGGL(cols, dim3(cus), dim3(K::WG1), lds1, 0, 8, maps, work, tw12);
           return hipGetLastError();
         }},
        {"ifft4096 cols_to_blocks one-shot", ib,
         [&] {
           hipLaunchKernelGGL(cols, dim3(8 * n / K::B), dim3(K::WG1), lds1, 0, 8, maps, work, tw12);
           return hipGetLastError();
         }},
        {"ifft4096 rows RPW 4 persistent", ib,
         [&] {
           hipLaunchKernelGGL(rows4, dim3(cus), dim3(K::WG2), twb + K::LDS2, 0, 8, g, work, maps, (float*)nullptr,
                              FoamParams{}, tw12);
           return hipGetLastError();
         }},
        {"ifft4096 rows RPW 4 one-shot", ib,
         [&] {
           hipLaunchKernelGGL(rows4, dim3(8 * n / 4), dim3(K::WG2), twb + K::LDS2, 0, 8, g, work, maps, (float*)nullptr,
                              FoamParams{}, tw12);
           return hipGetLastError();
         }},
        {"ifft4096 rows RPW 2 persistent (2/CU)", ib,
         [&] {
           hipLaunchKernelGGL(rows2, dim3(2 * cus), dim3(2 * S::T), lds2, 0, 8, g, work, maps, (float*)nullptr,
                              FoamParams{}, tw12);
           return hipGetLastError();
         }},
        {"ifft4096 rows RPW 2 one-shot", ib,
         [&] {
           hipLaunchKernelGGL(rows2, dim3(8 * n / 2), dim3(2 * S::T), lds2, 0, 8, g, work, maps, (float*)nullptr,
                              FoamParams{}, tw12);
           return hipGetLastError();
         }},
    };
    run_cases(ci, 7, 5);
    CHECK(hipFree(work));
    CHECK(hipFree(maps));
    CHECK(hipFree(tw12));
  }
  {
    // in-place EncodeIFFT passes at 8192 (4 images) and 16384 (1 image)
    for (int logn : {13, 14})
    {
      const int n = 1 << logn, imgs = logn == 13 ? 4 : 1;
      const size_t tex = (size_t)n * n * imgs;
      float4* img;
      CHECK(hipMalloc(&img, tex * 16));
      CHECK(hipMemset(img, 0, tex * 16));
      float2* tw = make_twiddles(logn);
      const double ib = 32.0 * tex;
      std::vector<Case> cr = {
          {std::to_string(n) + " rows in place persistent", ib,
           [&] { return persist([&] { return launch_rows_ifft(logn, imgs, img, tw, 0, cus); }); }},
          {std::to_string(n) + " rows in place one-shot", ib, [&] { return launch_rows_ifft(logn, imgs, img, tw, 0, BIG); }},
          {std::to_string(n) + " cols in place persistent", ib, [&] { return persist([&] { return launch_cols(logn, imgs, img, tw, 0, cus); }); }},
          {std::to_string(n) + " cols in place one-shot", ib, [&] { return launch_cols(logn, imgs, img, tw, 0, BIG); }},
      };
      run_cases(cr, 5, 3);
      CHECK(hipFree(img));
      CHECK(hipFree(tw));
    }
  }
  {
    // 16384^2 strip-dealt whole grid (P = 1): transposes + RM row pass, persistent vs one-shot
    const int logn = 14, n = 1 << logn, C = 1;
    const HalfSlab hsl{0, half_strips(logn), half_strips(logn), n};
    const size_t blk = half_slab_block_bytes(logn, C, hsl), rt = half_slab_row_texels(logn, C, n);
    unsigned char* recv;
    float4 *rab, *rde, *maps;
    float2* rc;
    float* jac;
    CHECK(hipMalloc(&recv, blk));
    CHECK(hipMemset(recv, 0, blk));
    CHECK(hipMalloc(&rab, rt * 16));
    CHECK(hipMalloc(&rde, rt * 16));
    CHECK(hipMalloc(&rc, rt * 8));
    CHECK(hipMalloc(&maps, (size_t)n * n * 2 * 16));
    CHECK(hipMalloc(&jac, (size_t)n * n * 4));
    float2* tw = make_twiddles(logn);
    float2* tw2 = make_twiddles(logn - 4);  // the XS row pass's N/16-point table
    FrameParams fp{};
    fp.cascades = 1;
    fp.c[0] = {2.0f * 3.14159265358f / 1000.0f, 37.5f, 9.8f, 100.0f};
    FoamParams foam{};
    foam.displacement[0] = 0.4f;
    const double pts = (double)n * n;
    std::vector<Case> cs = {
        {"16384 transposes + rows persistent (round-1 default)", 96.0 * pts,
         [&] { return persist([&] { return launch_half_slab_rows(logn, fp, hsl, recv, rab, rde, rc, maps, jac, foam, tw, tw2, 0, cus); }); }},
        {"16384 transposes + rows one-shot", 96.0 * pts,
         [&] { return launch_half_slab_rows(logn, fp, hsl, recv, rab, rde, rc, maps, jac, foam, tw, tw2, 0, BIG); }},
    };
    run_cases(cs, 5, 3);
  }
  return 0;
}
