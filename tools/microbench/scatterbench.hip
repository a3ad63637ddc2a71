// scatterbench.hip — can the XCD's L2 assemble whole lines from 16-byte column pieces written (or read)
// by different workgroups at the same time? One workgroup (1024 threads) moves one column of a
// row-major [R][K] float4 image (R = 16384 rows, 16 B per row); `group` consecutive columns are given
// to workgroups of one XCD that run concurrently (blocks b, b+8, ... under round-robin placement), so
// a 128-B line is covered by 8 workgroups' pieces. Compared with contiguous streams of the same bytes.
#include "all_kernels.h"

#include <cstdio>
#include <cstdlib>

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

__device__ __forceinline__ void ntst(float4 v, float4* p)
{
  __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(p));
}

constexpr int R = 16384, K = 8192, WG = 1024, PER = R / WG;

// block -> column for iteration `it`: `group` consecutive columns on `group` blocks of one XCD
__device__ __forceinline__ int column_of(int b, int G, int group, int it)
{
  const int xcd = b & 7, idx = b >> 3, per_xcd = G >> 3;
  const int groups_per_xcd = per_xcd / group;
  const int gid = xcd * groups_per_xcd + idx / group;
  return (it * (G / group) + gid) * group + idx % group;
}

// one column per item: write 16384 x 16 B at stride K*16 (NT: non-temporal stores)
template <bool NT, int W>
__global__ __launch_bounds__(WG) void k_colwrite(float4* __restrict__ img, int group)
{
  const int G = gridDim.x;
  for (int it = 0; it * G < K / W; it++)
  {
    const int col = column_of(blockIdx.x, G, group, it) * W;
#pragma unroll
    for (int m = 0; m < PER; m++)
    {
      const int row = m * WG + threadIdx.x;
#pragma unroll
      for (int w = 0; w < W; w++)
      {
        float4* p = img + (size_t)row * K + col + w;
        const float4 v = make_float4(row, col, w, 1.0f);
        if (NT)
          ntst(v, p);
        else
          *p = v;
      }
    }
  }
}

// one column per item: read 16384 x 16 B at stride K*16, write them contiguously to out
template <int W>
__global__ __launch_bounds__(WG) void k_colread(const float4* __restrict__ img, float4* __restrict__ out, int group)
{
  const int G = gridDim.x;
  for (int it = 0; it * G < K / W; it++)
  {
    const int col = column_of(blockIdx.x, G, group, it) * W;
    float4 v[PER * W];
#pragma unroll
    for (int m = 0; m < PER; m++)
#pragma unroll
      for (int w = 0; w < W; w++)
        v[m * W + w] = img[(size_t)(m * WG + threadIdx.x) * K + col + w];
    float4* o = out + (size_t)col * R;
#pragma unroll
    for (int m = 0; m < PER * W; m++)
      ntst(v[m], o + m * WG + threadIdx.x);
  }
}

__global__ __launch_bounds__(WG) void k_contig_write(float4* __restrict__ img, long n4)
{
  for (long i = (long)blockIdx.x * WG + threadIdx.x; i < n4; i += (long)gridDim.x * WG)
    ntst(make_float4(i, 0, 0, 1), img + i);
}

__global__ __launch_bounds__(WG) void k_contig_copy(const float4* __restrict__ a, float4* __restrict__ b, long n4)
{
  for (long i = (long)blockIdx.x * WG + threadIdx.x; i < n4; i += (long)gridDim.x * WG)
    ntst(a[i], b + i);
}

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
  return ms / reps;
}

int main()
{
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const long n4 = (long)R * K;  // 2 GiB of float4
  const double bytes = n4 * 16.0;
  float4 *a, *b;
  CHECK(hipMalloc(&a, n4 * 16));
  CHECK(hipMalloc(&b, n4 * 16));
  CHECK(hipMemset(a, 0, n4 * 16));
  CHECK(hipMemset(b, 0, n4 * 16));
  auto rep = [&](const char* name, double moved, float ms) {
    std::printf("%-58s %7.3f ms %7.1f GB/s\n", name, ms, moved / ms / 1e6);
  };
  rep("contiguous write (2 GiB)", bytes, time_ms([&] { hipLaunchKernelGGL(k_contig_write, dim3(cus * 2), dim3(WG), 0, 0, a, n4); }, 5));
  rep("contiguous copy (read + write)", 2 * bytes, time_ms([&] { hipLaunchKernelGGL(k_contig_copy, dim3(cus * 2), dim3(WG), 0, 0, a, b, n4); }, 5));
  const int G = cus;  // one 1024-thread block per CU
  char name[128];
  for (int group : {1, 2, 4, 8, 16, 32})
  {
    std::snprintf(name, sizeof name, "column write 16 B pieces, group %2d, default policy", group);
    rep(name, bytes, time_ms([&] { hipLaunchKernelGGL((k_colwrite<false, 1>), dim3(G), dim3(WG), 0, 0, a, group); }, 5));
    std::snprintf(name, sizeof name, "column write 16 B pieces, group %2d, nt", group);
    rep(name, bytes, time_ms([&] { hipLaunchKernelGGL((k_colwrite<true, 1>), dim3(G), dim3(WG), 0, 0, a, group); }, 5));
  }
  for (int group : {1, 4, 8})
  {
    std::snprintf(name, sizeof name, "column write 32 B pieces, group %2d, default policy", group);
    rep(name, bytes, time_ms([&] { hipLaunchKernelGGL((k_colwrite<false, 2>), dim3(G), dim3(WG), 0, 0, a, group); }, 5));
  }
  for (int group : {1, 2, 4, 8, 16})
  {
    std::snprintf(name, sizeof name, "column read 16 B pieces + contiguous write, group %2d", group);
    rep(name, 2 * bytes, time_ms([&] { hipLaunchKernelGGL((k_colread<1>), dim3(G), dim3(WG), 0, 0, a, b, group); }, 5));
  }
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  return 0;
}
