// copybench.hip — which streaming forms reach the HBM ceiling on gfx950 (out-of-place copies of
// 2 GiB float4, read + write counted). Variants: plain pointer vs buffer (SRD) access, unroll depth,
// cache-policy aux bits on the buffer loads/stores, workgroup size.
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

template <int UNROLL>
__global__ __launch_bounds__(256) void k_copy_ptr(const float4* __restrict__ a, float4* __restrict__ b, long n4)
{
  const long stride = (long)gridDim.x * 256 * UNROLL;
  for (long base = (long)blockIdx.x * 256 * UNROLL + threadIdx.x; base < n4; base += stride)
  {
    float4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++)
      v[u] = a[base + u * 256];
#pragma unroll
    for (int u = 0; u < UNROLL; u++)
      b[base + u * 256] = v[u];
  }
}

template <int UNROLL, int LAUX, int SAUX, int WG>
__global__ __launch_bounds__(WG) void k_copy_srd(const float4* __restrict__ a, float4* __restrict__ b, long n4)
{
  const long chunk = (long)WG * UNROLL;  // texels per block iteration
  for (long base = (long)blockIdx.x * chunk; base < n4; base += (long)gridDim.x * chunk)
  {
    __amdgpu_buffer_rsrc_t ra = srd(a + base, kAllBytes), rb = srd(b + base, kAllBytes);
    f4v v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++)
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, (threadIdx.x + u * WG) * 16, 0, LAUX);
#pragma unroll
    for (int u = 0; u < UNROLL; u++)
      __builtin_amdgcn_raw_buffer_store_b128(v[u], rb, (threadIdx.x + u * WG) * 16, 0, SAUX);
  }
}

// one-shot grids (no persistent loop): each thread copies PER float4 at stride WG, block b owns
// texels [b * WG * PER, (b + 1) * WG * PER); NT: non-temporal loads and stores
template <int PER, int WG, bool NT>
__global__ __launch_bounds__(WG) void k_copy_oneshot(const float4* __restrict__ a, float4* __restrict__ b)
{
  const long base = (long)blockIdx.x * WG * PER + threadIdx.x;
  f4v v[PER];
#pragma unroll
  for (int u = 0; u < PER; u++)
    v[u] = NT ? __builtin_nontemporal_load(reinterpret_cast<const f4v*>(a) + base + u * WG)
              : reinterpret_cast<const f4v*>(a)[base + u * WG];
#pragma unroll
  for (int u = 0; u < PER; u++)
  {
    if (NT)
      __builtin_nontemporal_store(v[u], reinterpret_cast<f4v*>(b) + base + u * WG);
    else
      reinterpret_cast<f4v*>(b)[base + u * WG] = v[u];
  }
}

// read-only: sum of PER float4 per thread, one store per block so nothing is optimised away
template <int PER, int WG>
__global__ __launch_bounds__(WG) void k_read_oneshot(const float4* __restrict__ a, float* __restrict__ out)
{
  const long base = (long)blockIdx.x * WG * PER + threadIdx.x;
  f4v acc = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < PER; u++)
    acc += __builtin_nontemporal_load(reinterpret_cast<const f4v*>(a) + base + u * WG);
  if (acc.x == 1234.5f)
    out[blockIdx.x] = acc.y;
}

template <int PER, int WG>
__global__ __launch_bounds__(WG) void k_write_oneshot(float4* __restrict__ b)
{
  const long base = (long)blockIdx.x * WG * PER + threadIdx.x;
#pragma unroll
  for (int u = 0; u < PER; u++)
    __builtin_nontemporal_store(f4v{1.0f, 2.0f, 3.0f, (float)u}, reinterpret_cast<f4v*>(b) + base + u * WG);
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
  const long n4 = 1L << 27;  // 2 GiB of float4
  float4 *a, *b;
  CHECK(hipMalloc(&a, n4 * 16));
  CHECK(hipMalloc(&b, n4 * 16));
  CHECK(hipMemset(a, 0, n4 * 16));
  CHECK(hipMemset(b, 0, n4 * 16));
  const double bytes = 2.0 * n4 * 16;
  auto rep = [&](const char* name, float ms) { std::printf("%-52s %7.3f ms %7.1f GB/s\n", name, ms, bytes / ms / 1e6); };
#define PTR(U, G)                                                                                                      \
  rep("ptr copy unroll " #U " grid " #G "/CU",                                                                         \
      time_ms([&] { hipLaunchKernelGGL(k_copy_ptr<U>, dim3(cus * G), dim3(256), 0, 0, a, b, n4); }, 10));
  PTR(1, 8) PTR(4, 8) PTR(4, 4) PTR(8, 4) PTR(16, 2)
#define SRD(U, LA, SA, WG, G)                                                                                          \
  rep("srd copy unroll " #U " laux " #LA " saux " #SA " wg " #WG " grid " #G "/CU",                                    \
      time_ms([&] { hipLaunchKernelGGL((k_copy_srd<U, LA, SA, WG>), dim3(cus * G), dim3(WG), 0, 0, a, b, n4); }, 10));
  SRD(4, 0, 0, 256, 8) SRD(16, 0, 0, 256, 4) SRD(16, 0, 0, 1024, 1) SRD(16, 0, 0, 512, 2)
  SRD(16, 2, 0, 256, 4) SRD(16, 0, 2, 256, 4) SRD(16, 2, 2, 256, 4) SRD(16, 1, 0, 256, 4) SRD(16, 0, 1, 256, 4)
  SRD(16, 3, 3, 256, 4) SRD(16, 2, 2, 1024, 1) SRD(16, 0, 2, 1024, 1)
#define ONE(PER, WG, NT)                                                                                               \
  rep("oneshot copy per " #PER " wg " #WG " nt " #NT,                                                                  \
      time_ms([&] { hipLaunchKernelGGL((k_copy_oneshot<PER, WG, NT>), dim3(n4 / (PER * WG)), dim3(WG), 0, 0, a, b); }, 10));
  ONE(1, 256, false) ONE(1, 256, true) ONE(4, 256, false) ONE(4, 256, true) ONE(8, 256, true) ONE(16, 256, true)
  ONE(4, 512, true) ONE(4, 1024, true) ONE(2, 256, true)
  {
    float* dummy;
    CHECK(hipMalloc(&dummy, 1 << 24));
    auto repo = [&](const char* name, double moved, float ms) { std::printf("%-52s %7.3f ms %7.1f GB/s\n", name, ms, moved / ms / 1e6); };
    repo("read-only nt per 4 wg 256", n4 * 16.0, time_ms([&] { hipLaunchKernelGGL((k_read_oneshot<4, 256>), dim3(n4 / 1024), dim3(256), 0, 0, a, dummy); }, 10));
    repo("read-only nt per 16 wg 256", n4 * 16.0, time_ms([&] { hipLaunchKernelGGL((k_read_oneshot<16, 256>), dim3(n4 / 4096), dim3(256), 0, 0, a, dummy); }, 10));
    repo("write-only nt per 4 wg 256", n4 * 16.0, time_ms([&] { hipLaunchKernelGGL((k_write_oneshot<4, 256>), dim3(n4 / 1024), dim3(256), 0, 0, b); }, 10));
    repo("write-only nt per 16 wg 256", n4 * 16.0, time_ms([&] { hipLaunchKernelGGL((k_write_oneshot<16, 256>), dim3(n4 / 4096), dim3(256), 0, 0, b); }, 10));
    CHECK(hipFree(dummy));
  }
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  return 0;
}
