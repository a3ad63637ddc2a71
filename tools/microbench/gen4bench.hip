// gen4bench.hip — the four-step whole-grid column pass at N = 16384 (k_gen4_step1 / k_gen4_step2):
// step 1 at several occupancy bounds and step 2 at 16 / 8 columns per workgroup, interleaved, with
// the production launchers' frame for reference. Outputs are compared with the production variant
// (bit-identical: same arithmetic, different launch shapes). Usage: gen4bench
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
  launch();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; r++)
    launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms / reps;
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

int main()
{
  constexpr int LOGN = 14, LOGN2 = 10;
  constexpr int N = 1 << LOGN;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int C = 1;
  float4* h0;
  CHECK(hipMalloc(&h0, (size_t)N * N * 16));
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
  s.planeSize = 1000;
  s.scale = 1;
  s.spread = 0.2f;
  CHECK(launch_generate_spectrum(s, N, h0, 0, cus, 0, 0, gen4_h0_block()));
  FrameParams fp{};
  fp.cascades = C;
  fp.c[0] = {2.0f * 3.14159265358f / s.planeSize, 37.5f, s.g, s.h};
  // whole grid (P = 1): step 1 into the parts, step 2 into the one exchange block
  const Gen4Geom g = gen4_geom(LOGN, C, 0, 1, true);
  const int KP = g.cols + g.nyq, PITCH = g.lp;
  unsigned char *buf, *blk;
  const size_t part = (size_t)C * N * PITCH;  // texels per part
  CHECK(hipMalloc(&buf, gen4_parts_bytes(LOGN, C, g)));
  CHECK(hipMalloc(&blk, g.blk_bytes));
  const size_t rt = (size_t)C * g.w * PITCH;  // texels per block field
  float2 *tw = table(LOGN), *tw2 = table(LOGN2);
  const int items1 = C * ((KP + 63) / 64) * (N / 64);
  auto s1 = [&](auto kern) {
    return [=] { hipLaunchKernelGGL(kern, dim3(items1), dim3(256), 0, 0, fp, g, h0, buf, tw); };
  };
  const float4* wab = reinterpret_cast<const float4*>(buf);
  auto s2 = [&](auto kp, auto kc, int ci) {
    const int lds = ((FftShape<LOGN2>::TW_ENTRIES * 8 + 15) / 16) * 16 + ci * FftShape<LOGN2>::PADDED * 8;
    CHECK(hipFuncSetAttribute((const void*)kp, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CHECK(hipFuncSetAttribute((const void*)kc, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    const int gpn = C * 16 * ((KP + ci - 1) / ci), gcn = C * 16 * (((KP + 1) / 2 + ci - 1) / ci);
    const int wg = FftShape<LOGN2>::T * ci;
    return [=] {
      hipLaunchKernelGGL(kp, dim3(gpn), dim3(wg), lds, 0, C, KP, PITCH, wab, blk, (size_t)0, g, tw2, (const uint64_t*)nullptr);
      hipLaunchKernelGGL(kp, dim3(gpn), dim3(wg), lds, 0, C, KP, PITCH, wab + part, blk, 16 * rt, g, tw2, (const uint64_t*)nullptr);
      hipLaunchKernelGGL(kc, dim3(gcn), dim3(wg), lds, 0, C, (KP + 1) / 2, PITCH / 2, wab + 2 * part, blk, 32 * rt, g, tw2, (const uint64_t*)nullptr);
    };
  };
  float4* rab = reinterpret_cast<float4*>(blk);
  struct V
  {
    std::string name;
    std::function<void()> run;
    double bytes;
    std::vector<float> t;
  };
  const double pts = (double)N * N;
  auto s1r2 = [&](auto kern) {
    return [=] { hipLaunchKernelGGL(kern, dim3(items1), dim3(256), 0, 0, fp, h0, buf, tw); };
  };
  std::vector<V> vs = {
      {"step 1, launch bound 1 (production)", s1(k_gen4_step1<LOGN, 1>), 28 * pts, {}},
      {"step 1 of round 2 (waterfall loads)", s1r2(k_gen4_step1_r2<LOGN, 1>), 28 * pts, {}},
      {"step 1, min 2 waves/SIMD", s1(k_gen4_step1<LOGN, 2>), 28 * pts, {}},
      {"step 1, min 3 waves/SIMD", s1(k_gen4_step1<LOGN, 3>), 28 * pts, {}},
      {"step 1, min 4 waves/SIMD", s1(k_gen4_step1<LOGN, 4>), 28 * pts, {}},
      {"step 2, 8 columns/WG, 2 WG/CU (production)", s2(k_gen4_step2<LOGN2, true, 8>, k_gen4_step2<LOGN2, false, 8>, 8), 40 * pts, {}},
      {"step 2, 16 columns/WG", s2(k_gen4_step2<LOGN2, true>, k_gen4_step2<LOGN2, false>, 16), 40 * pts, {}},
      {"step 2, 4 columns/WG", s2(k_gen4_step2<LOGN2, true, 4>, k_gen4_step2<LOGN2, false, 4>, 4), 40 * pts, {}},
  };
  // identity: each variant's output vs the first of its step
  auto snap = [&](const void* p, size_t n) {
    std::vector<unsigned char> h(n);
    CHECK(hipMemcpy(h.data(), p, n, hipMemcpyDeviceToHost));
    return h;
  };
  vs[0].run();
  CHECK(hipDeviceSynchronize());
  auto ref1 = snap(buf, 40 * part);
  for (int k = 1; k < 5; k++)
  {
    CHECK(hipMemset(buf, 0, 40 * part));
    vs[k].run();
    CHECK(hipDeviceSynchronize());
    std::printf("%s: parts %s\n", vs[k].name.c_str(), snap(buf, 40 * part) == ref1 ? "bit-identical" : "DIFFER");
  }
  vs[5].run();
  CHECK(hipDeviceSynchronize());
  auto ref2 = snap(rab, rt * 16);
  for (int k = 6; k < 8; k++)
  {
    CHECK(hipMemset(rab, 0, rt * 16));
    vs[k].run();
    CHECK(hipDeviceSynchronize());
    std::printf("%s: block gab %s\n", vs[k].name.c_str(), snap(rab, rt * 16) == ref2 ? "bit-identical" : "DIFFER");
  }
  for (int r = 0; r < 5; r++)
    for (auto& v : vs)
      v.t.push_back(time_ms(v.run, 3));
  for (auto& v : vs)
  {
    std::sort(v.t.begin(), v.t.end());
    std::printf("%-40s median %7.3f ms  %7.1f GB/s algorithmic\n", v.name.c_str(), v.t[2], v.bytes / v.t[2] / 1e6);
  }
  return 0;
}
