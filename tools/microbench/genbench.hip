// genbench.hip — interleaved A/B timing of the generator frame passes (8 cascades x 4096^2).
// Build: see Makefile target `microbench`.
#include "all_kernels.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
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

int main(int argc, char** argv)
{
  const int logn = argc > 1 ? std::atoi(argv[1]) : 12;
  const int C = argc > 2 ? std::atoi(argv[2]) : 8;
  const int n = 1 << logn;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t tex = (size_t)n * n;
  float4 *h0, *inter, *maps;
  float* jac;
  float2* tw;
  CHECK(hipMalloc(&h0, tex * C * sizeof(float4)));
  CHECK(hipMalloc(&inter, tex * C * 2 * sizeof(float4)));
  CHECK(hipMalloc(&maps, tex * C * 2 * sizeof(float4)));
  CHECK(hipMalloc(&jac, tex * C * sizeof(float)));
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
    fp.c[c] = {2.0f * 3.14159265358f / s.planeSize, 1.0f, s.g, s.h};
    foam.displacement[c] = s.displacement;
  }
  CHECK(hipDeviceSynchronize());
  const double pts = (double)tex * C;
  SlabGeom geom{0, n};
  float4* scratch = nullptr;
  if (rows_need_transpose(logn))
    CHECK(hipMalloc(&scratch, tex * C * 2 * sizeof(float4)));
  // half-spectrum path buffers (N = 1024 .. 4096)
  float4 *gab = nullptr, *gcd = nullptr, *spec = nullptr;
  float2* ge = nullptr;
  const bool half = half_spectrum_supported(logn);
  if (half)
  {
    const size_t ht = half_field_texels(logn) * C;
    CHECK(hipMalloc(&gab, ht * sizeof(float4)));
    CHECK(hipMalloc(&gcd, ht * sizeof(float4)));
    CHECK(hipMalloc(&ge, ht * sizeof(float2)));
    CHECK(hipMalloc(&spec, (size_t)C * 2 * n * sizeof(float4)));
  }
  auto h1 = [&] { return launch_half_columns_ab(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus); };
  auto h2 = [&] { return launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus); };
  auto p1r = [&] { return launch_cols_evolve(logn, fp, geom, h0, inter, tw, 0, cus, 0); };
  auto p1k = [&] { return launch_cols_evolve(logn, fp, geom, h0, inter, tw, 0, cus, 16); };
  auto p1h = [&] { return launch_cols_evolve(logn, fp, geom, h0, inter, tw, 0, cus, default_keep(logn)); };
  auto p2 = [&] { return launch_rows_final(logn, C, geom, inter, scratch, maps, jac, foam, tw, 0, cus); };
  auto pv = [&](int pass, int pol) {
    return [&, pass, pol] {
      return pass == 1 ? launch_policy_variant(1, pol, fp, geom, h0, inter, nullptr, foam, tw, 0, cus)
                       : launch_policy_variant(2, pol, fp, geom, inter, maps, jac, foam, tw, 0, cus);
    };
  };
  auto frame = [&] {
    hipError_t e = p1h();
    return e == hipSuccess ? p2() : e;
  };
  (void)p1r(); (void)p1k(); (void)p1h(); (void)p2();
  CHECK(hipDeviceSynchronize());
  const int rounds = 7, reps = 10;
  std::vector<float> t1r, t1k, t1h, t2, tf;
  std::vector<std::vector<float>> tp(6);
  std::vector<float> tco, trp2, t2c, t2m, t1m, th1, th2;
  for (int r = 0; r < rounds; r++)
  {
    t1r.push_back(time_ms(p1r, reps));
    t1k.push_back(time_ms(p1k, reps));
    t1h.push_back(time_ms(p1h, reps));
    t2.push_back(time_ms(p2, reps));
    tf.push_back(time_ms(frame, reps));
    if (logn == 12)
      for (int pass = 1; pass <= 2; pass++)
        for (int pol = 0; pol < 3; pol++)
          tp[(pass - 1) * 3 + pol].push_back(time_ms(pv(pass, pol), reps));
    if (logn == 12)
    {
      tco.push_back(time_ms(pv(1, 3), reps));
      trp2.push_back(time_ms(pv(2, 3), reps));
      t2c.push_back(time_ms(pv(2, 4), reps));
      t2m.push_back(time_ms(pv(2, 5), reps));
      t1m.push_back(time_ms(pv(1, 4), reps));
      th1.push_back(time_ms(h1, reps));
      th2.push_back(time_ms(h2, reps));
    }
  }
  auto report = [&](const char* name, std::vector<float>& v, double bytes_per_pt) {
    std::sort(v.begin(), v.end());
    std::printf("%-34s median %7.3f ms  min %7.3f ms  %7.1f GB/s (algorithmic %.0f B/pt)\n", name, v[v.size() / 2],
                v[0], bytes_per_pt * pts / v[v.size() / 2] / 1e6, bytes_per_pt);
  };
  std::printf("N=%d cascades=%d CUs=%d\n", n, C, cus);
  report("pass1 cols_evolve (re-read h0)", t1r, 48);
  report("pass1 cols_evolve (keep 16 H)", t1k, 48);
  report("pass1 cols_evolve (default keep)", t1h, 48);
  report("pass2 rows_final", t2, 68);
  report("frame (pass1 default keep + pass2)", tf, 116);
  if (logn == 12)
  {
    const char* pn[2][3] = {{"keep 0 reread default", "keep 4 reread default", "keep 4 all loads default"}, {"policy default", "policy nt stores", "policy nt loads+stores"}};
    for (int pass = 1; pass <= 2; pass++)
      for (int pol = 0; pol < 3; pol++)
      {
        char name[80];
        std::snprintf(name, sizeof name, "pass%d %s", pass, pn[pass - 1][pol]);
        report(name, tp[(pass - 1) * 3 + pol], pass == 1 ? 48 : 68);
      }
    report("pass1 keep 4 compute only (no HBM)", tco, 48);
    report("pass2 2 rows per WG (2 WG/CU)", trp2, 68);
    report("pass2 compute only (no HBM)", t2c, 68);
    report("pass2 memory only (no FFT)", t2m, 68);
    report("pass1 keep 4 memory only (no evolve/FFT)", t1m, 48);
    report("half pass1 (Nyquist term + k_cols_half)", th1, 28);
    report("half pass2 k_rows_half (both images per item)", th2, 56);
    for (int a = 1; a <= 5; a++)
    {
      static const char* names[] = {"", "half pass2 no HBM loads", "half pass2 no FFT", "half pass2 no mirror exchange",
                                    "half pass2 4 rows per WG (1 WG/CU)", "half pass2 1 row per WG (4 WG/CU)"};
      auto ha = [&] { return launch_half_rows_ab(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus, a); };
      std::vector<float> ta;
      for (int r = 0; r < rounds; r++)
        ta.push_back(time_ms(ha, reps));
      report(names[a], ta, 56);
    }
  }
  return 0;
}
