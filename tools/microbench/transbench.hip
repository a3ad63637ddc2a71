// transbench.hip — tile shapes for the strip-dealt path's field transpose at N = 16384, B = 1:
// in [strip][row] (8193 strips x 16384 rows of float4, strip-major) -> out [row][strip] (row-major).
// Each tile is TU strips x TY rows through LDS; reads are TY-texel runs per strip, writes TU-texel
// runs per row. BATCH: all loads issued before the LDS writes.
#include "all_kernels.h"

#include <cstdio>
#include <cstdlib>

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

using oceanfft::f4v;
constexpr int W = 16384, KP = 8193;

// PADS: texels of padding per strip (strip stride W + PADS): a power-of-two stride (256 KiB) may put
// every strip of a tile on the same HBM channel
template <int TU, int TY, int WG, bool BATCH, int PADS = 0, bool NT = false>
__global__ __launch_bounds__(WG) void k_trans(const float4* __restrict__ in, float4* __restrict__ out)
{
  constexpr int PER = TU * TY / WG;
  __shared__ float4 tile[TU][TY + 1];
  const int tiles_u = (KP + TU - 1) / TU, tiles_y = W / TY;
  for (int item = blockIdx.x; item < tiles_u * tiles_y; item += gridDim.x)
  {
    const int tu = item % tiles_u, ty = item / tiles_u;
    float4 v[PER];
#pragma unroll
    for (int k = 0; k < PER; k++)
    {
      const int L = k * WG + threadIdx.x, row = L % TY, st = L / TY, u = tu * TU + st;
      float4 x = make_float4(0, 0, 0, 0);
      if (u < KP)
      {
        const float4* p = in + (size_t)u * (W + PADS) + ty * TY + row;
        if (NT)
        {
          const f4v t = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
          x = make_float4(t.x, t.y, t.z, t.w);
        }
        else
          x = *p;
      }
      if (BATCH)
        v[k] = x;
      else
        tile[st][row] = x;
    }
    if (BATCH)
    {
#pragma unroll
      for (int k = 0; k < PER; k++)
      {
        const int L = k * WG + threadIdx.x, row = L % TY, st = L / TY;
        tile[st][row] = v[k];
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; k++)
    {
      const int L = k * WG + threadIdx.x, col = L % TU, row = L / TU;
      if (tu * TU + col < KP)
      {
        float4* p = out + (size_t)(ty * TY + row) * KP + tu * TU + col;
        const float4 t = tile[col][row];
        if (NT)
          __builtin_nontemporal_store(f4v{t.x, t.y, t.z, t.w}, reinterpret_cast<f4v*>(p));
        else
          *p = t;
      }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_copy(const float4* __restrict__ a, float4* __restrict__ b, long n)
{
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    b[i] = a[i];
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
  const long n = (long)(W + 256) * KP;
  float4 *a, *b;
  CHECK(hipMalloc(&a, n * 16));
  CHECK(hipMalloc(&b, n * 16));
  CHECK(hipMemset(a, 0, n * 16));
  const double bytes = 2.0 * n * 16;
  auto rep = [&](const char* name, float ms) { std::printf("%-44s %7.3f ms %7.1f GB/s\n", name, ms, bytes / ms / 1e6); };
#define T(TU, TY, WG, BATCH, G)                                                                                       \
  rep("tile " #TU "x" #TY " wg " #WG " batch " #BATCH " grid " #G "/CU",                                              \
      time_ms([&] { hipLaunchKernelGGL((k_trans<TU, TY, WG, BATCH>), dim3(cus * G), dim3(WG), 0, 0, a, b); }, 5));
  rep("contiguous copy", time_ms([&] { hipLaunchKernelGGL(k_copy, dim3(cus * 8), dim3(256), 0, 0, a, b, n); }, 5));
  rep("contiguous copy one-shot", time_ms([&] { hipLaunchKernelGGL(k_copy, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, a, b, n); }, 5));
  T(128, 32, 256, true, 64)
  T(64, 64, 256, true, 64)
#define TP(TU, TY, PADS)                                                                                              \
  rep("tile " #TU "x" #TY " strip stride W + " #PADS, time_ms([&] {                                                 \
        hipLaunchKernelGGL((k_trans<TU, TY, 256, true, PADS>), dim3(cus * 4), dim3(256), 0, 0, a, b); }, 5));
  TP(128, 32, 0) TP(128, 32, 8) TP(128, 32, 32) TP(128, 32, 64) TP(128, 32, 136) TP(64, 64, 8) TP(64, 64, 72)
  TP(256, 16, 8) TP(256, 16, 72)
#define TN(TU, TY, NT, G)                                                                                             \
  rep("tile " #TU "x" #TY " nt " #NT " grid " #G "/CU", time_ms([&] {                                               \
        hipLaunchKernelGGL((k_trans<TU, TY, 256, true, 0, NT>), dim3(cus * G), dim3(256), 0, 0, a, b); }, 5));
  TN(128, 32, true, 4) TN(256, 16, false, 4) TN(256, 16, true, 4) TN(512, 8, false, 4) TN(512, 8, true, 4)
  TN(256, 8, true, 8) TN(512, 4, true, 8) TN(1024, 4, true, 4)
  T(64, 64, 256, false, 4)
  T(64, 64, 256, true, 4)
  T(64, 64, 256, true, 2)
  T(32, 128, 256, true, 4)
  T(16, 256, 256, true, 4)
  T(128, 32, 256, true, 4)
  T(32, 64, 256, true, 8)
  T(64, 32, 256, true, 8)
  T(32, 32, 256, true, 16)
  T(64, 64, 512, true, 2)
  T(64, 64, 512, false, 2)
  T(32, 64, 256, false, 8)
  {
    // the production kernel on the same shape (P = 1, strips = KP, w = W)
    oceanfft::HalfSlab h{0, KP, KP, W};
    const size_t blk = (size_t)KP * W * 16;
    rep("production k_half_to_rows<float4, 1> grid 4/CU", time_ms([&] {
          hipLaunchKernelGGL((oceanfft::k_half_to_rows<float4, 1>), dim3(cus * 4), dim3(256), 0, 0, 1, 16384, h,
                             (const unsigned char*)a, (size_t)0, blk, b);
        }, 5));
    const int tiles = ((KP + 127) / 128) * (W / 32);  // one block per tile (no persistent loop)
    rep("production k_half_to_rows<float4, 1> one-shot", time_ms([&] {
          hipLaunchKernelGGL((oceanfft::k_half_to_rows<float4, 1>), dim3(tiles), dim3(256), 0, 0, 1, 16384, h,
                             (const unsigned char*)a, (size_t)0, blk, b);
        }, 5));
    rep("production k_half_to_rows<float4, 1> grid 8/CU", time_ms([&] {
          hipLaunchKernelGGL((oceanfft::k_half_to_rows<float4, 1>), dim3(cus * 8), dim3(256), 0, 0, 1, 16384, h,
                             (const unsigned char*)a, (size_t)0, blk, b);
        }, 5));
  }
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  return 0;
}
