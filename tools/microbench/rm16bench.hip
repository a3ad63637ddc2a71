// rm16bench.hip — the row pass of whole 16384^2 grids (k_rows_half, RM layout, one row of both
// images per 1024-thread item): the plain x transform (14 barriers per image) against XS (the
// four-step x transform with per-wave sub-transforms, 6 barriers), with timing ablations: no HBM
// loads (ABL 1), no x transform (ABL 2). Ablated outputs are wrong by construction. Builds with
// -DOCEAN_ABLATE_EXCHANGE / -DOCEAN_ABLATE_BARRIER price the exchanges and barriers.
// Usage: rm16bench
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

__global__ void fill(float* p, size_t n, unsigned salt)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
  {
    unsigned h = (unsigned)i * 2654435761u ^ salt;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    p[i] = ((float)(h & 0xffff) - 32768.0f) * (1.0f / 32768.0f);
  }
}

// lane_xchg.h check: element e = 64 m + lane; after transpose_reg_lanes_2_5 the value at (m, lane) must
// be the element whose register bits 0..3 and lane bits 2..5 are exchanged; after the two permlane
// swaps (register bits 2, 3 <-> lane bits 4, 5) likewise. Counts mismatches.
__global__ void k_check_lane_xchg(int* bad)
{
  const int lane = threadIdx.x;
  CPair v[16], u[16];
  for (int m = 0; m < 16; m++)
  {
    const float e = (float)(64 * m + lane);
    v[m] = CPair{f2v{e, e + 0.25f}, f2v{e + 0.5f, e + 0.75f}};
    u[m] = v[m];
  }
  transpose_reg_lanes_2_5(v);
  swap_reg_lane_bit<2, 4>(u);
  swap_reg_lane_bit<3, 5>(u);
  int nb = 0;
  for (int m = 0; m < 16; m++)
  {
    const int om = (lane >> 2) & 15, ol = (lane & 3) | (m << 2);  // full 4 x 4 transposition
    const float e = (float)(64 * om + ol);
    nb += v[m].re.x != e || v[m].re.y != e + 0.25f || v[m].im.x != e + 0.5f || v[m].im.y != e + 0.75f;
    const int pm = (m & 3) | (((lane >> 4) & 3) << 2), pl = (lane & 15) | (((m >> 2) & 3) << 4);
    const float f = (float)(64 * pm + pl);
    nb += u[m].re.x != f || u[m].im.y != f + 0.75f;
  }
  atomicAdd(bad, nb);
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
  constexpr int LOGN = 14;
  using S = FftShape<LOGN>;
  constexpr int N = 1 << LOGN, PITCH = N / 2 + 16;  // the four-step path's row pitch at P = 1
  const int C = 1;
  const size_t rt = (size_t)N * PITCH;
  float4 *rab, *rde, *spec, *maps;
  float2* rc;
  float* jac;
  CHECK(hipMalloc(&rab, rt * 16));
  CHECK(hipMalloc(&rde, rt * 16));
  CHECK(hipMalloc(&rc, rt * 8));
  CHECK(hipMalloc(&spec, (size_t)2 * N * 16));
  CHECK(hipMalloc(&maps, (size_t)2 * N * N * 16));
  CHECK(hipMalloc(&jac, (size_t)N * N * 4));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (float*)rab, rt * 4, 1u);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (float*)rde, rt * 4, 2u);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (float*)rc, rt * 2, 3u);
  hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, 0, (float*)spec, (size_t)2 * N * 4, 4u);
  CHECK(hipDeviceSynchronize());
  FrameParams fp{};
  fp.cascades = C;
  fp.c[0] = {2.0f * 3.14159265358f / 1000.0f, 37.5f, 9.8f, 100.0f};
  FoamParams foam{};
  foam.displacement[0] = 0.4f;
  float2* tw = table(LOGN);
  float2* tw2 = table(LOGN - 4);
  const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + lds_row_slots<LOGN>(1) * 8;
  const RowSrc rs{reinterpret_cast<const unsigned char*>(rab), reinterpret_cast<const unsigned char*>(rde),
                  reinterpret_cast<const unsigned char*>(rc), 0, N / 2, PITCH, 0};
  auto mk = [&](auto kern, int per = 1) {
    CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    return [=] {
      hipLaunchKernelGGL(kern, dim3(C * N * per), dim3(S::T), lds, 0, fp, rab, rde, rc, spec, maps, jac, foam, tw, N,
                         rs, (const float2*)nullptr);
    };
  };
  struct V
  {
    std::string name;
    std::function<void()> run;
    std::vector<float> t;
  };
  auto mkx = [&](auto kern) {
    CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, XsCfg<LOGN>::LDS));
    return [=] {
      hipLaunchKernelGGL(kern, dim3(C * N), dim3(S::T), XsCfg<LOGN>::LDS, 0, fp, rab, rde, rc, spec, maps, jac, foam, tw,
                         N, rs, tw2);
    };
  };
  auto mkn = [&](auto kern) {  // k_rows_xs (spec, maps, jac, foam, tw, rows, rs, tw2)
    CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, XsCfg<LOGN>::LDS));
    return [=] {
      hipLaunchKernelGGL(kern, dim3(C * N), dim3(S::T), XsCfg<LOGN>::LDS, 0, fp, spec, maps, jac, foam, tw, N, rs, tw2);
    };
  };
  auto mkg = [&](auto kern, int grid) {  // k_rows_xs on a persistent grid: PF prefetches the next row too
    CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, XsCfg<LOGN>::LDS));
    return [=] {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(S::T), XsCfg<LOGN>::LDS, 0, fp, spec, maps, jac, foam, tw, N, rs, tw2);
    };
  };
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  auto mkp = [&](auto kern) {  // k_rows_xp (spec, maps, jac, foam, tw, rows, rs)
    CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, XpCfg<LOGN>::LDS));
    return [=] {
      hipLaunchKernelGGL(kern, dim3(C * N), dim3(S::T), XpCfg<LOGN>::LDS, 0, fp, spec, maps, jac, foam, tw, N, rs);
    };
  };
  {
    int* bad;
    CHECK(hipMalloc(&bad, 4));
    CHECK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(k_check_lane_xchg, dim3(1), dim3(64), 0, 0, bad);
    int hb = -1;
    CHECK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
    std::printf("lane_xchg check: %d mismatching values%s\n", hb, hb ? " (WRONG)" : " (exact)");
    CHECK(hipFree(bad));
  }
  std::vector<V> vs = {
      {"row pass, plain transform (round 2)", mk(k_rows_half<LOGN, kStream, kStream, 0, 1, true, true>), {}},
      {"XS (four-step x transform)", mkx(k_rows_half<LOGN, kStream, kStream, 0, 1, true, true, 1, 1, 4, 2, true, true>), {}},
      {"XS, default-policy loads", mkx(k_rows_half<LOGN, 0, kStream, 0, 1, true, true, 1, 1, 4, 2, true, true>), {}},
      {"XS ABL 1: no HBM loads", mkx(k_rows_half<LOGN, kStream, kStream, 1, 1, true, true, 1, 1, 4, 2, true, true>), {}},
      {"ABL 1: no HBM loads", mk(k_rows_half<LOGN, kStream, kStream, 1, 1, true, true>), {}},
      {"ABL 2: no x transform", mk(k_rows_half<LOGN, kStream, kStream, 2, 1, true, true>), {}},
      {"k_rows_xs (C loaded per image)", mkn(k_rows_xs<LOGN, 0>), {}},
      {"k_rows_xs, 2 of 8 loads prefetched", mkn(k_rows_xs<LOGN, 2>), {}},
      {"k_rows_xs, 3 of 8 loads prefetched", mkn(k_rows_xs<LOGN, 3>), {}},
      {"k_rows_xs PF 2, block index by division (before)", mkn(k_rows_xs_div<LOGN, 2>), {}},
      {"k_rows_xp (64 x 256, permlane/DPP), PF 0", mkp(k_rows_xp<LOGN, 0>), {}},
      {"k_rows_xp PF 2", mkp(k_rows_xp<LOGN, 2>), {}},
      {"k_rows_xp PF 3", mkp(k_rows_xp<LOGN, 3>), {}},
      {"k_rows_xs_r3 (round-3 production) PF 2", mkn(k_rows_xs_r3<LOGN, 2>), {}},
      {"k_rows_xs PF 2, persistent grid (CUs)", mkg(k_rows_xs<LOGN, 2>, cus), {}},
      {"k_rows_xs PF 3, persistent grid (CUs)", mkg(k_rows_xs<LOGN, 3>, cus), {}},
      {"k_rows_xs PF 0, persistent grid (CUs)", mkg(k_rows_xs<LOGN, 0>, cus), {}},
      {"k_rows_xs PF 2 EARLY 1", mkn(k_rows_xs<LOGN, 2, 1>), {}},
      {"k_rows_xs PF 2 EARLY 2", mkn(k_rows_xs<LOGN, 2, 2>), {}},
      {"k_rows_xs PF 0 EARLY 1", mkn(k_rows_xs<LOGN, 0, 1>), {}},
      {"k_rows_xs PF 0 EARLY 2", mkn(k_rows_xs<LOGN, 0, 2>), {}},
      {"k_rows_xs EARLY 3, persistent grid (CUs)", mkg(k_rows_xs<LOGN, 0, 3>, cus), {}},
      {"k_rows_xs EARLY 3, one-shot grid", mkn(k_rows_xs<LOGN, 0, 3>), {}},
      {"k_rows_xs PF 0 EARLY 2, persistent grid (CUs)", mkg(k_rows_xs<LOGN, 0, 2>, cus), {}},
      {"k_rows_xs EARLY 4 (C kept for image 1), persistent", mkg(k_rows_xs<LOGN, 0, 4>, cus), {}},
  };
  // XS vs the plain transform: same lanes, different rounding order (max |diff| vs max |value|)
  auto snapf = [&](const void* p, size_t n) {
    std::vector<float> h(n / 4);
    CHECK(hipMemcpy(h.data(), p, n, hipMemcpyDeviceToHost));
    return h;
  };
  const size_t mb = (size_t)2 * N * N * 16, jb = (size_t)N * N * 4;
  auto compare = [&](int a, int b, const char* what) {
    vs[a].run();
    CHECK(hipDeviceSynchronize());
    const auto m0 = snapf(maps, mb), j0 = snapf(jac, jb);
    CHECK(hipMemset(maps, 0, mb));
    CHECK(hipMemset(jac, 0, jb));
    vs[b].run();
    CHECK(hipDeviceSynchronize());
    const auto m1 = snapf(maps, mb), j1 = snapf(jac, jb);
    double dm = 0, am = 0, dj = 0, aj = 0;
    for (size_t k = 0; k < m0.size(); k++)
    {
      dm = std::max(dm, (double)std::fabs(m0[k] - m1[k]));
      am = std::max(am, (double)std::fabs(m0[k]));
    }
    for (size_t k = 0; k < j0.size(); k++)
    {
      dj = std::max(dj, (double)std::fabs(j0[k] - j1[k]));
      aj = std::max(aj, (double)std::fabs(j0[k]));
    }
    std::printf("%s: maps max|diff| %.3g of max|v| %.3g; jac %.3g of %.3g%s\n", what, dm, am, dj, aj,
                m0 == m1 && j0 == j1 ? " (bit-identical)" : "");
  };
  compare(0, 1, "XS vs plain");
  compare(1, 6, "k_rows_xs vs XS");
  compare(1, 7, "k_rows_xs PF 2 vs XS");
  compare(1, 8, "k_rows_xs PF 3 vs XS");
  compare(7, 9, "k_rows_xs PF 2: shift vs division");
  compare(1, 2, "XS streamed vs default-policy loads");
  compare(7, 10, "k_rows_xp PF 0 vs k_rows_xs PF 2");
  compare(7, 11, "k_rows_xp PF 2 vs k_rows_xs PF 2");
  compare(10, 12, "k_rows_xp PF 3 vs PF 0");
  compare(13, 7, "k_rows_xs PF 2 (streaming T_in) vs round 3");
  compare(7, 14, "k_rows_xs PF 2: persistent vs one-shot grid");
  compare(7, 17, "k_rows_xs PF 2 EARLY 1 vs PF 2");
  compare(7, 18, "k_rows_xs PF 2 EARLY 2 vs PF 2");
  compare(7, 19, "k_rows_xs PF 0 EARLY 1 vs PF 2");
  compare(7, 20, "k_rows_xs PF 0 EARLY 2 vs PF 2");
  compare(7, 21, "k_rows_xs EARLY 3 persistent vs PF 2");
  compare(7, 22, "k_rows_xs EARLY 3 one-shot vs PF 2");
  compare(7, 23, "k_rows_xs PF 0 EARLY 2 persistent vs PF 2");
  compare(7, 24, "k_rows_xs EARLY 4 persistent vs PF 2");
  for (int r = 0; r < 5; r++)
    for (auto& v : vs)
      v.t.push_back(time_ms(v.run, 3));
  const double bytes = 56.04 * (double)N * N;
  for (auto& v : vs)
  {
    std::sort(v.t.begin(), v.t.end());
    std::printf("%-32s median %7.3f ms  %7.1f GB/s at 56 B/pt\n", v.name.c_str(), v.t[2], bytes / v.t[2] / 1e6);
  }
  return 0;
}
