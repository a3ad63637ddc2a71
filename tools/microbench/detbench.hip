// detbench.hip — run-twice determinism of the frame passes: the same inputs through the production
// launchers twice (and a third time after other work), every output compared bit for bit. Built twice
// (Makefile): detbench (production buffer helpers) and detbench_soffset (-DOCEAN_SOFFSET_PIECES: the
// piece offsets of ld4s / st4s / ld2s / st2s in the SGPR soffset field, the round-2 build whose
// fields differed between runs; DESIGN.md §3 "Register budget").
// Usage: detbench [reps]
#include "all_kernels.h"

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

static std::vector<unsigned char> snap(const void* d, size_t bytes)
{
  std::vector<unsigned char> h(bytes);
  CHECK(hipMemcpy(h.data(), d, bytes, hipMemcpyDeviceToHost));
  return h;
}

static size_t differing(const std::vector<unsigned char>& a, const std::vector<unsigned char>& b)
{
  const float* x = reinterpret_cast<const float*>(a.data());
  const float* y = reinterpret_cast<const float*>(b.data());
  size_t d = 0;
  for (size_t k = 0; k < a.size() / 4; k++)
    d += std::memcmp(x + k, y + k, 4) != 0;
  return d;
}

static float2* table(int logn)
{
  const int n = 1 << logn, lb = logn / 2, tb = 1 << lb, ta = 1 << (logn - lb);
  std::vector<float2> tab(tb + ta);
  for (int e = 0; e < tb; e++)
    tab[e] = make_float2((float)std::cos(2 * M_PI * e / n), (float)std::sin(2 * M_PI * e / n));
  for (int e = 0; e < ta; e++)
    tab[tb + e] = make_float2((float)std::cos(2 * M_PI * (double)e * tb / n), (float)std::sin(2 * M_PI * (double)e * tb / n));
  float2* d;
  CHECK(hipMalloc(&d, tab.size() * 8));
  CHECK(hipMemcpy(d, tab.data(), tab.size() * 8, hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv)
{
  const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
  const int logn = 12, n = 1 << logn, C = 8;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t tex = (size_t)n * n, ht = half_field_texels(logn) * C;
  float4 *h0, *gab, *gcd, *spec, *maps;
  float2 *ge, *hs;
  float* jac;
  CHECK(hipMalloc(&h0, tex * C * 16));
  CHECK(hipMalloc(&gab, ht * 16));
  CHECK(hipMalloc(&gcd, ht * 16));
  CHECK(hipMalloc(&ge, ht * 8));
  CHECK(hipMalloc(&spec, (size_t)C * 2 * n * 16));
  CHECK(hipMalloc(&hs, half_hs_bytes(logn, cus)));
  CHECK(hipMalloc(&maps, tex * C * 32));
  CHECK(hipMalloc(&jac, tex * C * 4));
  float2* tw = table(logn);
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
    s.planeSize = planes[c];
    s.scale = 1;
    s.spread = 0.2f;
    CHECK(launch_generate_spectrum(s, n, h0 + tex * c, 0, cus));
    fp.c[c] = {2.0f * 3.14159265358f / s.planeSize, 37.5f, s.g, s.h};
    foam.displacement[c] = s.displacement;
  }
  auto frame = [&] {
    CHECK(launch_half_columns(logn, fp, h0, gab, gcd, ge, spec, tw, 0, cus, hs, cus));
    CHECK(launch_half_rows(logn, fp, gab, gcd, ge, spec, maps, jac, foam, tw, 0, cus));
    CHECK(hipDeviceSynchronize());
  };
  frame();
  const auto f0 = snap(gab, ht * 16), f1 = snap(gcd, ht * 16), f2 = snap(ge, ht * 8), m0 = snap(maps, tex * C * 32);
  size_t worst = 0;
  for (int r = 0; r < reps; r++)
  {
    CHECK(hipMemset(gab, 0, ht * 16));
    CHECK(hipMemset(hs, 0xff, half_hs_bytes(logn, cus)));  // a stale scratch must not leak into the fields
    frame();
    const size_t d = differing(f0, snap(gab, ht * 16)) + differing(f1, snap(gcd, ht * 16)) +
                     differing(f2, snap(ge, ht * 8)) + differing(m0, snap(maps, tex * C * 32));
    std::printf("%s run %d: %zu differing floats (fields + maps of 8 x 4096^2)\n",
#if defined(OCEAN_SOFFSET_PIECES)
                "soffset pieces",
#else
                "production (voffset pieces)",
#endif
                r + 1, d);
    worst = d > worst ? d : worst;
  }
  std::printf("%s\n", worst == 0 ? "DETERMINISTIC" : "NON-DETERMINISTIC");
  return 0;
}
