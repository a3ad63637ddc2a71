// transbench.hip — tile shapes for the strip-dealt path's field transpose at N = 16384, B = 1:
// in [strip][row] (8193 strips x 16384 rows of float4, strip-major) -> out [row][strip] (row-major).
// Each tile is TU strips x TY rows through LDS; reads are TY-texel runs per strip, writes TU-texel
// runs per row. BATCH: all loads issued before the LDS writes.
#include "../../oceansimulation_amd/csrc/ocean_kernels.hip"

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

constexpr int W = 16384, KP = 8193;

template <int TU, int TY, int WG, bool BATCH>
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
        x = in[(size_t)u * W + ty * TY + row];
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
        out[(size_t)(ty * TY + row) * KP + tu * TU + col] = tile[col][row];
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
  const long n = (long)W * KP;
  float4 *a, *b;
  CHECK(hipMalloc(&a, n * 16));
  CHECK(hipMalloc(&b, n * 16));
  CHECK(hipMemset(a, 0, n * 16));
  const double bytes = 2.0 * n * 16;
  auto rep = [&](const char* name, float ms) { std::printf("%-44s %7.3f ms %7.1f GB/s\n", name, ms, bytes / ms / 1e6); };
  rep("contiguous copy", time_ms([&] { hipLaunchKernelGGL(k_copy, dim3(cus * 8), dim3(256), 0, 0, a, b, n); }, 5));
#define T(TU, TY, WG, BATCH, G)                                                                                       \
  rep("tile " #TU "x" #TY " wg " #WG " batch " #BATCH " grid " #G "/CU",                                              \
      time_ms([&] { hipLaunchKernelGGL((k_trans<TU, TY, WG, BATCH>), dim3(cus * G), dim3(WG), 0, 0, a, b); }, 5));
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
  }
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  return 0;
}
