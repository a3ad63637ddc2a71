// valubench.hip — VALU issue rates on gfx950 for the FFT's arithmetic forms: scalar v_fma_f32 /
// v_add_f32 against packed v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32 (the split-plane CPair
// butterflies), 16 waves per CU (1024-thread blocks), 8 independent chains per thread.
// Reports lane-operations per second (a packed instruction counts 2 per lane).
#include <hip/hip_runtime.h>

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

typedef float f2v __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096, CH = 8;

template <int KIND>
__global__ __launch_bounds__(1024) void k_valu(float* out, float s)
{
  float a[CH];
  f2v p[CH];
  for (int c = 0; c < CH; c++)
  {
    a[c] = threadIdx.x * 1e-3f + c;
    p[c] = f2v{a[c], a[c] + 0.5f};
  }
  const float m = s, k = 1.0f - s;
  const f2v mm = {m, m}, kk = {k, k};
  for (int it = 0; it < ITERS; it++)
  {
#pragma unroll
    for (int c = 0; c < CH; c++)
    {
      if constexpr (KIND == 0)  // v_fma_f32
        a[c] = __builtin_fmaf(a[c], m, k);
      else if constexpr (KIND == 1)  // v_add_f32
        a[c] = a[c] + m;
      else if constexpr (KIND == 2)  // v_pk_fma_f32
        p[c] = __builtin_elementwise_fma(p[c], mm, kk);
      else if constexpr (KIND == 3)  // v_pk_add_f32
        p[c] = p[c] + mm;
      else  // v_pk_mul_f32
        p[c] = p[c] * mm;
    }
  }
  float r = 0;
  for (int c = 0; c < CH; c++)
    r += KIND < 2 ? a[c] : p[c].x + p[c].y;
  if (r == 1234.5f)
    out[threadIdx.x] = r;
}

int main()
{
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float* out;
  CHECK(hipMalloc(&out, 4096));
  const char* names[] = {"v_fma_f32", "v_add_f32", "v_pk_fma_f32", "v_pk_add_f32", "v_pk_mul_f32"};
  for (int rep = 0; rep < 2; rep++)
    for (int kind = 0; kind < 5; kind++)
    {
      hipEvent_t a, b;
      CHECK(hipEventCreate(&a));
      CHECK(hipEventCreate(&b));
      auto launch = [&] {
        switch (kind)
        {
        case 0: hipLaunchKernelGGL(k_valu<0>, dim3(cus * 2), dim3(1024), 0, 0, out, 0.999f); break;
        case 1: hipLaunchKernelGGL(k_valu<1>, dim3(cus * 2), dim3(1024), 0, 0, out, 0.999f); break;
        case 2: hipLaunchKernelGGL(k_valu<2>, dim3(cus * 2), dim3(1024), 0, 0, out, 0.999f); break;
        case 3: hipLaunchKernelGGL(k_valu<3>, dim3(cus * 2), dim3(1024), 0, 0, out, 0.999f); break;
        default: hipLaunchKernelGGL(k_valu<4>, dim3(cus * 2), dim3(1024), 0, 0, out, 0.999f); break;
        }
      };
      launch();
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(a));
      launch();
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms;
      CHECK(hipEventElapsedTime(&ms, a, b));
      const double insts = (double)cus * 2 * 1024 / 64 * ITERS * CH;  // wave-instructions
      const double lanes = (kind >= 2 ? 2.0 : 1.0) * insts * 64;
      const double per_simd = insts / (cus * 4);
      if (rep == 1)
        std::printf("%-14s %8.3f ms  %7.2f cycles/wave-instr/SIMD at 2.4 GHz  %8.1f T lane-ops/s\n", names[kind], ms,
                    ms * 1e-3 * 2.4e9 / per_simd, lanes / ms / 1e9);
    }
  return 0;
}
