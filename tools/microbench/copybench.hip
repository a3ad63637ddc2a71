// copybench.hip — which streaming forms reach the HBM ceiling on gfx950 (out-of-place copies of
// 2 GiB float4, read + write counted). Variants: plain pointer vs buffer (SRD) access, unroll depth,
// cache-policy aux bits on the buffer loads/stores, workgroup size.
#include "../../oceansimulation_amd/csrc/ocean_kernels.hip"

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
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  return 0;
}
