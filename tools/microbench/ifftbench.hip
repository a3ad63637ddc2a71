// ifftbench.hip — the standalone EncodeIFFT's strided column pass (k_cols_to_blocks, 8 packed 4096^2
// images read in 64-B row pieces) under load cache policy x XCD grouping of adjacent strips, and the
// row pass that follows, timed interleaved in one process. Output checked identical across variants.
#include "all_kernels.h"

#include <algorithm>
#include <cstring>
#include <functional>
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
    launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main()
{
  constexpr int LOGN = 12, N = 1 << LOGN, IMG = 8;
  using K = ColFirstCfg<LOGN>;
  using S = FftShape<LOGN>;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t tex = (size_t)N * N * IMG;
  float4 *img, *work, *ref;
  CHECK(hipMalloc(&img, tex * 16));
  CHECK(hipMalloc(&work, tex * 16));
  CHECK(hipMalloc(&ref, tex * 16));
  std::vector<float4> h(tex);
  for (size_t k = 0; k < tex; k++)
    h[k] = make_float4(std::sin(0.001 * k), std::cos(0.0007 * k), 0.5f, -0.25f);
  CHECK(hipMemcpy(img, h.data(), tex * 16, hipMemcpyHostToDevice));
  int lb = LOGN / 2, tb = 1 << lb, ta = 1 << (LOGN - lb);
  std::vector<float2> tab(tb + ta);
  for (int e = 0; e < tb; e++)
    tab[e] = make_float2((float)std::cos(2 * M_PI * e / N), (float)std::sin(2 * M_PI * e / N));
  for (int e = 0; e < ta; e++)
    tab[tb + e] = make_float2((float)std::cos(2 * M_PI * e * tb / N), (float)std::sin(2 * M_PI * e * tb / N));
  float2* tw;
  CHECK(hipMalloc(&tw, tab.size() * sizeof(float2)));
  CHECK(hipMemcpy(tw, tab.data(), tab.size() * sizeof(float2), hipMemcpyHostToDevice));
  const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + K::LDS1;

  auto launch = [&](auto kern) {
    CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    // one block per strip (the production one-shot grid)
    return [=] { hipLaunchKernelGGL(kern, dim3(IMG * (N / K::B)), dim3(K::WG1), lds, 0, IMG, img, work, tw); };
  };
  struct V
  {
    const char* name;
    std::function<void()> run;
  };
  std::vector<V> vs = {
      {"default loads, pairs (production)", launch(k_cols_to_blocks<LOGN, 0, 2>)},
      {"nt loads, pairs", launch(k_cols_to_blocks<LOGN, kStream, 2>)},
      {"nt loads, no grouping", launch(k_cols_to_blocks<LOGN, kStream, 1>)},
      {"nt loads, groups of 4", launch(k_cols_to_blocks<LOGN, kStream, 4>)},
      {"default loads, groups of 4", launch(k_cols_to_blocks<LOGN, 0, 4>)},
      {"nt loads, groups of 8", launch(k_cols_to_blocks<LOGN, kStream, 8>)},
      {"default loads, groups of 8", launch(k_cols_to_blocks<LOGN, 0, 8>)},
  };
  vs[0].run();
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(ref, work, tex * 16, hipMemcpyDeviceToDevice));
  std::vector<float4> a(tex), b(tex);
  CHECK(hipMemcpy(a.data(), ref, tex * 16, hipMemcpyDeviceToHost));
  for (auto& v : vs)
  {
    CHECK(hipMemset(work, 0, tex * 16));
    v.run();
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(b.data(), work, tex * 16, hipMemcpyDeviceToHost));
    if (std::memcmp(a.data(), b.data(), tex * 16) != 0)
      std::printf("MISMATCH: %s\n", v.name);
  }
  std::vector<std::vector<float>> t(vs.size());
  for (int r = 0; r < 7; r++)
    for (size_t k = 0; k < vs.size(); k++)
      t[k].push_back(time_ms(vs[k].run, 5));
  const double bytes = 32.0 * tex;
  for (size_t k = 0; k < vs.size(); k++)
  {
    std::sort(t[k].begin(), t[k].end());
    std::printf("%-40s median %6.3f ms  %7.1f GB/s\n", vs[k].name, t[k][3], bytes / t[k][3] / 1e6);
  }
  return 0;
}
