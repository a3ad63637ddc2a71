// layoutbench.hip — memory-only floors of the two frame passes for intermediate block widths
// BOUT = 4 (current: pass 1 writes whole 64-B block rows, pass 2 reads 256-B runs) and BOUT = 8
// (pass 1 writes 64-B halves of 128-B block rows, two workgroups per block paired on one XCD;
// pass 2 reads 512-B runs). No arithmetic: loads, stores and the same lane maps as the kernels.
// 8 cascades x 4096^2, h0 16 B/pt, intermediate 32 B/pt, maps 32 B/pt + Jacobian 4 B/pt.
#include "all_kernels.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

constexpr int N = 4096, T = 256, C = 8;

// pass-1 pattern: item = 4-column strip of one cascade; h0 [c][xb4][y][4] read contiguously;
// output [c][img][x / BOUT][y][BOUT]. PAIR: strips 2k and 2k+1 (one 128-B block row) go to
// blocks b and b+8 (same XCD under round-robin dispatch).
template <int BOUT, bool PAIR>
__global__ __launch_bounds__(1024) void k_p1(const float4* __restrict__ h0, float4* __restrict__ inter)
{
  const int strips = N / 4, total = C * strips;
  const int G = gridDim.x;
  for (int it = PAIR ? xcd_pair_slot(blockIdx.x, G) : blockIdx.x; it < total; it += G)
  {
    const int tid = opaque((int)threadIdx.x);
    const int b = tid % 4, i = tid / 4;
    const int c = it / strips, xb4 = it % strips;
    const float4* src = h0 + ((size_t)c * strips + xb4) * N * 4;
    float4 v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
      v[m] = ld4<kStream>(src + m * T * 4, (i * 4 + b) * 16);
    const int x = xb4 * 4 + b, xo = x / BOUT, bo = x % BOUT;
#pragma unroll
    for (int img = 0; img < 2; img++)
    {
      float4* dst = inter + ((size_t)(c * 2 + img) * (N / BOUT) + xo) * N * BOUT;
#pragma unroll
      for (int m = 0; m < 16; m++)
      {
        float4 o = v[m];
        o.x += img;
        st4<kStream>(dst + m * T * BOUT, (i * BOUT + bo) * 16, o);
      }
    }
  }
}

// pass-2 pattern: item = RPW rows of one image; loads lanes (b fastest, then r, then ihi) from
// [c][img][xb][y][BOUT]: 16*BOUT/... one BOUT*RPW*16-byte run per BOUT*RPW lanes; stores the rows
// row-major with i fastest, plus a Jacobian float for odd images.
template <int BOUT>
__global__ __launch_bounds__(1024) void k_p2(const float4* __restrict__ inter, float4* __restrict__ maps,
                                             float* __restrict__ jac)
{
  constexpr int RPW = 4;
  const int blocks = N / RPW, total = C * 2 * blocks;
  for (int it = blockIdx.x; it < total; it += gridDim.x)
  {
    const int tid = opaque((int)threadIdx.x);
    const int b = tid % BOUT, r = (tid / BOUT) % RPW, ihi = tid / (BOUT * RPW);
    const int cimg = it / blocks, y0 = (it % blocks) * RPW;
    const float4* src = inter + (size_t)cimg * N * N + (size_t)y0 * BOUT;
    float4 v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
      v[m] = ld4<kStream>(src + (size_t)(m * (T / BOUT)) * N * BOUT, ((ihi * N + r) * BOUT + b) * 16);
    const int i2 = tid % T, r2 = tid / T;
    float4* dst = maps + ((size_t)cimg * N + y0) * N;
#pragma unroll
    for (int m = 0; m < 16; m++)
      st4<kStream>(dst + m * T, ((r2 * N) + i2) * 16, v[m]);
    if (cimg & 1)
    {
      float* jb = jac + ((size_t)(cimg >> 1) * N + y0) * N;
#pragma unroll
      for (int m = 0; m < 16; m++)
        st1<kStream>(jb + m * T, ((r2 * N) + i2) * 4, v[m].y * v[m].z);
    }
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
  const size_t pts = (size_t)C * N * N;
  float4 *h0, *inter, *maps;
  float* jac;
  CHECK(hipMalloc(&h0, pts * 16));
  CHECK(hipMalloc(&inter, pts * 32));
  CHECK(hipMalloc(&maps, pts * 32));
  CHECK(hipMalloc(&jac, pts * 4));
  CHECK(hipMemset(h0, 0, pts * 16));
  CHECK(hipMemset(inter, 0, pts * 32));
  const int grid = cus;  // one 1024-thread workgroup per CU, as the frame kernels
  std::vector<float> t[5];
  for (int round = 0; round < 7; round++)
  {
    t[0].push_back(time_ms([&] { hipLaunchKernelGGL((k_p1<4, false>), dim3(grid), dim3(1024), 0, 0, h0, inter); }, 10));
    t[1].push_back(time_ms([&] { hipLaunchKernelGGL((k_p1<8, true>), dim3(grid), dim3(1024), 0, 0, h0, inter); }, 10));
    t[2].push_back(time_ms([&] { hipLaunchKernelGGL((k_p1<8, false>), dim3(grid), dim3(1024), 0, 0, h0, inter); }, 10));
    t[3].push_back(time_ms([&] { hipLaunchKernelGGL((k_p2<4>), dim3(grid), dim3(1024), 0, 0, inter, maps, jac); }, 10));
    t[4].push_back(time_ms([&] { hipLaunchKernelGGL((k_p2<8>), dim3(grid), dim3(1024), 0, 0, inter, maps, jac); }, 10));
  }
  const char* names[] = {"pass1 pattern BOUT 4", "pass1 pattern BOUT 8 paired on XCD", "pass1 pattern BOUT 8 unpaired",
                         "pass2 pattern BOUT 4 (256-B runs)", "pass2 pattern BOUT 8 (512-B runs)"};
  const double bytes[] = {48, 48, 48, 68, 68};
  for (int k = 0; k < 5; k++)
  {
    std::sort(t[k].begin(), t[k].end());
    const float med = t[k][t[k].size() / 2];
    std::printf("%-40s median %7.3f ms  %7.1f GB/s\n", names[k], med, bytes[k] * pts / med / 1e6);
  }
  return 0;
}
