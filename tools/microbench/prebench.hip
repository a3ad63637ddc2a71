// prebench.hip — standalone EncodeIFFT at N = 8192 / 16384: the production orders (8192: column-first
// through a work image with two-column items; 16384: rows + the four-step column transform through a
// work slab) against the radix-R pre-stage column pass (k_cols_pre: 4-column strips, R = N / 4096
// items per strip, each a 4096-point transform) with its row pass, work layouts WL 0 (blocked,
// permuted rows) and 1 (row-major). Each result is compared with the in-place rows + columns
// (relative max error per image). Usage: prebench [images]
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

static float2* upload(const std::vector<float2>& t)
{
  float2* d;
  CHECK(hipMalloc(&d, t.size() * 8));
  CHECK(hipMemcpy(d, t.data(), t.size() * 8, hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv)
{
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int imgs = argc > 1 ? std::atoi(argv[1]) : 2;
  const int only = argc > 2 ? std::atoi(argv[2]) : 0;  // 12, 13 or 14: that size only
  for (int logn : {12, 13, 14})
  {
    if (only ? logn != only : logn == 12)
      continue;
    const int n = 1 << logn;
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
    CHECK(hipMalloc(&work, tex * 16));
    float2 *twn = upload(table(logn)), *tw2 = upload(table(logn - 4)), *twm = upload(table(12));
    CHECK(hipMemcpy(ref, h.data(), tex * 16, hipMemcpyHostToDevice));
    CHECK(launch_rows_ifft(logn, imgs, ref, twn, 0, cus));
    CHECK(launch_cols(logn, imgs, ref, twn, 0, cus));
    CHECK(hipDeviceSynchronize());
    std::vector<float4> a(tex), b(tex);
    CHECK(hipMemcpy(a.data(), ref, tex * 16, hipMemcpyDeviceToHost));

    std::vector<std::string> names;
    std::vector<std::function<hipError_t()>> runs;
    if (logn == 12)
    {
      // 4096: the column-first production (4-row row items, one 1024-thread workgroup per CU, streamed
      // loads) against fewer rows per item (more workgroups per CU) and default-policy row loads
      names.push_back("production: column-first, 4-row row items");
      runs.push_back([&] { return launch_ifft_colfirst(12, imgs, img, work, twn, 0, cus); });
      names.push_back("4-row row items, default-policy row loads");
      runs.push_back([&] { return launch_ifft_colfirst_ab<12, 2, 1, 4, 0>(imgs, img, work, twn, 0, cus); });
      names.push_back("2-row row items (512 threads)");
      runs.push_back([&] { return launch_ifft_colfirst_ab<12, 2, 1, 2>(imgs, img, work, twn, 0, cus); });
      names.push_back("2-row row items, default-policy row loads");
      runs.push_back([&] { return launch_ifft_colfirst_ab<12, 2, 1, 2, 0>(imgs, img, work, twn, 0, cus); });
      names.push_back("1-row row items (256 threads), pairs per line");
      runs.push_back([&] { return launch_ifft_colfirst_ab<12, 2, 2, 1>(imgs, img, work, twn, 0, cus); });
      names.push_back("1-row row items, pairs per line, default-policy row loads");
      runs.push_back([&] { return launch_ifft_colfirst_ab<12, 2, 2, 1, 0>(imgs, img, work, twn, 0, cus); });
    }
    else if (logn == 13)
    {
      names.push_back("production: column-first (2-column items) + blocked rows");
      runs.push_back([&] { return launch_ifft_colfirst(13, imgs, img, work, twn, 0, cus); });
      names.push_back("pre-stage R=2, WL 0 (blocked, permuted rows)");
      runs.push_back([&] { return launch_ifft_pre_t<13, 0>(imgs, img, work, twn, twm, 0, cus); });
      names.push_back("pre-stage R=2, WL 1 (row-major work)");
      runs.push_back([&] { return launch_ifft_pre_t<13, 1>(imgs, img, work, twn, twm, 0, cus); });
      names.push_back("pre-stage R=2, WL 0, streamed column loads");
      runs.push_back([&] { return launch_ifft_pre_t<13, 0, kStream>(imgs, img, work, twn, twm, 0, cus); });
      names.push_back("pre-stage R=2, WL 0, default-policy row loads");
      runs.push_back([&] { return launch_ifft_pre_t<13, 0, 0, 0>(imgs, img, work, twn, twm, 0, cus); });
      names.push_back("pre-stage R=2, WL 0, one-row row items (GRPR 2)");
      runs.push_back([&] { return launch_ifft_pre_t<13, 0, 0, kStream, 1>(imgs, img, work, twn, twm, 0, cus); });
      names.push_back("pre-stage R=2, WL 0, one-row row items, default-policy row loads");
      runs.push_back([&] { return launch_ifft_pre_t<13, 0, 0, 0, 1>(imgs, img, work, twn, twm, 0, cus); });
      names.push_back("pre-stage R=2, WL 0, column loads in batches of 4 points");
      runs.push_back([&] { return launch_ifft_pre_t<13, 0, 0, kStream, 2, 4>(imgs, img, work, twn, twm, 0, cus); });
      names.push_back("pre-stage R=2, WL 0, column loads in batches of 1 point");
      runs.push_back([&] { return launch_ifft_pre_t<13, 0, 0, kStream, 2, 1>(imgs, img, work, twn, twm, 0, cus); });
    }
    else
    {
      names.push_back("production: rows + four-step columns (wc 2048)");
      runs.push_back([&] { return launch_ifft_fourstep(14, imgs, img, work, 2048, twn, tw2, 0, cus); });
      names.push_back("pre-stage R=4, WL 0 (blocked, permuted rows)");
      runs.push_back([&] { return launch_ifft_pre_t<14, 0>(imgs, img, work, twn, twm, 0, cus); });
      names.push_back("pre-stage R=4, WL 1 (row-major work)");
      runs.push_back([&] { return launch_ifft_pre_t<14, 1>(imgs, img, work, twn, twm, 0, cus); });
      names.push_back("pre-stage R=4, residue pairs on 2-column strips");
      runs.push_back([&] { return launch_ifft_pre_pair14<0>(imgs, img, work, twn, twm, 0, cus); });
      names.push_back("pre-stage R=4, residue pairs, streamed row loads");
      runs.push_back([&] { return launch_ifft_pre_pair14<kStream>(imgs, img, work, twn, twm, 0, cus); });
    }
    // the four-step slab uses `work` as its slab (N x 2048 texels fit in the image-sized buffer)
    for (size_t k = 0; k < runs.size(); k++)
    {
      CHECK(hipMemcpy(img, h.data(), tex * 16, hipMemcpyHostToDevice));
      CHECK(runs[k]());
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemcpy(b.data(), img, tex * 16, hipMemcpyDeviceToHost));
      double mx = 0, er = 0;
      for (size_t q = 0; q < tex; q++)
        for (int j = 0; j < 4; j++)
        {
          mx = std::max(mx, (double)std::fabs((&a[q].x)[j]));
          er = std::max(er, (double)std::fabs((&a[q].x)[j] - (&b[q].x)[j]));
        }
      std::printf("N=%d x%d %-58s vs in-place max |diff| / max |x| = %.3g\n", n, imgs, names[k].c_str(), er / mx);
    }
    std::vector<std::vector<float>> t(runs.size());
    for (int rep = 0; rep < 7; rep++)
      for (size_t k = 0; k < runs.size(); k++)
        t[k].push_back(time_ms(runs[k], 3));
    for (size_t k = 0; k < runs.size(); k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::printf("N=%d x%d %-58s median %7.3f ms  %6.0f GB/s at 64 B/texel\n", n, imgs, names[k].c_str(), t[k][3],
                  64.0 * (double)tex / t[k][3] / 1e6);
    }
    CHECK(hipFree(img));
    CHECK(hipFree(ref));
    CHECK(hipFree(work));
  }
  return 0;
}
