// sqcontrol.hip — SQ-counter controls for the frame kernels: streaming kernels
// with the frame kernels' occupancy, timed and profiled with the same counter sets (tools/pmc_sq.sh
// passes, run on this binary), so the kernels' issue-stall / wait shares have a reference point.
//   copy_1024x1: 1024-thread workgroups, one per CU (80 KiB of LDS each), 16 float4 per thread per
//                iteration, nt loads and stores: the row pass's occupancy with no compute at all;
//   copy_256x4:  256-thread workgroups, four per CU: the k_rows_hp occupancy;
//   xpose_1024x1: as copy_1024x1 but every iteration goes load -> LDS -> barrier -> transposed read
//                -> store: the phase structure (one workgroup per CU, memory and LDS phases in turn)
//                of the FFT passes without their arithmetic.
// 2 GiB read + 2 GiB written per launch; prints ms and GB/s (read + write).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "device/memory.h"

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

template <int WG, bool XPOSE>
__device__ __forceinline__ void stream_body(const float4* __restrict__ a, float4* __restrict__ b, long n4)
{
  extern __shared__ __attribute__((aligned(16))) float4 lds[];
  constexpr int U = 16;
  const long chunk = (long)WG * U;
  for (long base = (long)blockIdx.x * chunk; base < n4; base += (long)gridDim.x * chunk)
  {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      v[u] = ld4<2>(a + base, (threadIdx.x + u * WG) * 16);
    if constexpr (XPOSE)
    {
      // one 64-KiB half at a time, as the FFT passes' split exchanges do (8 B slots, two halves)
#pragma unroll
      for (int h = 0; h < 2; h++)
      {
        __syncthreads();
        float2* x = reinterpret_cast<float2*>(lds);
#pragma unroll
        for (int u = 0; u < U; u++)
          x[u * WG + threadIdx.x] = h ? make_float2(v[u].z, v[u].w) : make_float2(v[u].x, v[u].y);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < U; u++)
        {
          const float2 t = x[threadIdx.x * U + (u ^ (threadIdx.x & 15))];
          if (h)
          {
            v[u].z = t.x;
            v[u].w = t.y;
          }
          else
          {
            v[u].x = t.x;
            v[u].y = t.y;
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      st4<2>(b + base, (threadIdx.x + u * WG) * 16, v[u]);
  }
}

template <int WG>
__global__ __launch_bounds__(WG) void k_stream_copy(const float4* __restrict__ a, float4* __restrict__ b, long n4)
{
  stream_body<WG, false>(a, b, n4);
}

__global__ __launch_bounds__(1024) void k_stream_xpose(const float4* __restrict__ a, float4* __restrict__ b, long n4)
{
  stream_body<1024, true>(a, b, n4);
}

template <typename F>
static float time_ms(F&& f, int reps)
{
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  f();
  CHECK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; r++)
    f();
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main()
{
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const long n4 = 1L << 27;  // 2 GiB of float4
  float4 *a, *b;
  CHECK(hipMalloc(&a, n4 * 16));
  CHECK(hipMalloc(&b, n4 * 16));
  CHECK(hipMemset(a, 0, n4 * 16));
  const double bytes = 2.0 * n4 * 16;
  const int big = 80 * 1024;  // one 1024-thread workgroup per CU
  CHECK(hipFuncSetAttribute((const void*)k_stream_copy<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, big));
  CHECK(hipFuncSetAttribute((const void*)k_stream_xpose, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
  float ms = time_ms([&] { hipLaunchKernelGGL((k_stream_copy<1024>), dim3(cus), dim3(1024), big, 0, a, b, n4); }, 10);
  std::printf("copy_1024x1   %7.3f ms %7.1f GB/s\n", ms, bytes / ms / 1e6);
  ms = time_ms([&] { hipLaunchKernelGGL((k_stream_copy<256>), dim3(cus * 4), dim3(256), 0, 0, a, b, n4); }, 10);
  std::printf("copy_256x4    %7.3f ms %7.1f GB/s\n", ms, bytes / ms / 1e6);
  ms = time_ms([&] { hipLaunchKernelGGL(k_stream_xpose, dim3(cus), dim3(1024), 128 * 1024, 0, a, b, n4); }, 10);
  std::printf("xpose_1024x1  %7.3f ms %7.1f GB/s\n", ms, bytes / ms / 1e6);
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  return 0;
}
