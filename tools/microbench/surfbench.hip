// surfbench.hip — the surface consumer (k_surface) against variants that load only
// the channels each stage uses and issue the normal stage's samples of all cascades together.
// Scene: 3 cascades of 256^2 random maps (L = 5 / 17 / 101 m, scale 1), the bench's camera, plane meshes
// of 1024^2 and 4096^2 quads. Every variant must reproduce k_surface bit for bit (same fp32 operations
// in the same order; only the loads and the loop structure differ).
// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -std=c++17 -I include -I oceansimulation_amd/csrc \
//        tools/microbench/surfbench.hip -o tools/microbench/surfbench
#include "all_kernels.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

namespace
{

// round 6's production sampler before the change: all four channels per tap (float4 loads)
template <int CH>
__device__ __forceinline__ void sample_linear_repeat(const float* __restrict__ tex, int n, float u, float v, float* out)
{
#pragma clang fp contract(off)
  const float s = u * (float)n - 0.5f, t = v * (float)n - 0.5f;
  const float fs = floorf(s), ft = floorf(t);
  const float a = s - fs, b = t - ft;
  const int m = n - 1;
  const int i0 = (int)fs & m, j0 = (int)ft & m, i1 = (i0 + 1) & m, j1 = (j0 + 1) & m;
  const float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
  const float* t00 = tex + ((size_t)j0 * n + i0) * CH;
  const float* t10 = tex + ((size_t)j0 * n + i1) * CH;
  const float* t01 = tex + ((size_t)j1 * n + i0) * CH;
  const float* t11 = tex + ((size_t)j1 * n + i1) * CH;
  if constexpr (CH == 4)
  {
    const float4 q00 = *reinterpret_cast<const float4*>(t00), q10 = *reinterpret_cast<const float4*>(t10);
    const float4 q01 = *reinterpret_cast<const float4*>(t01), q11 = *reinterpret_cast<const float4*>(t11);
    out[0] = w00 * q00.x + w10 * q10.x + w01 * q01.x + w11 * q11.x;
    out[1] = w00 * q00.y + w10 * q10.y + w01 * q01.y + w11 * q11.y;
    out[2] = w00 * q00.z + w10 * q10.z + w01 * q01.z + w11 * q11.z;
    out[3] = w00 * q00.w + w10 * q10.w + w01 * q01.w + w11 * q11.w;
  }
  else
    out[0] = w00 * t00[0] + w10 * t10[0] + w01 * t01[0] + w11 * t11[0];
}

// the four taps and weights of one GL_LINEAR + GL_REPEAT sample
struct Taps
{
  int o00, o10, o01, o11;  // texel indices
  float w00, w10, w01, w11;
};

__device__ __forceinline__ Taps taps_of(int n, float u, float v)
{
#pragma clang fp contract(off)
  const float s = u * (float)n - 0.5f, t = v * (float)n - 0.5f;
  const float fs = floorf(s), ft = floorf(t);
  const float a = s - fs, b = t - ft;
  const int m = n - 1;
  const int i0 = (int)fs & m, j0 = (int)ft & m, i1 = (i0 + 1) & m, j1 = (j0 + 1) & m;
  return Taps{j0 * n + i0, j0 * n + i1, j1 * n + i0, j1 * n + i1, (1.0f - a) * (1.0f - b), a * (1.0f - b),
              (1.0f - a) * b, a * b};
}

// channel ch of a map of CH floats per texel
template <int CH>
__device__ __forceinline__ float tap_sum(const float* __restrict__ tex, const Taps& k, int ch)
{
#pragma clang fp contract(off)
  const float q00 = tex[k.o00 * CH + ch], q10 = tex[k.o10 * CH + ch], q01 = tex[k.o01 * CH + ch],
              q11 = tex[k.o11 * CH + ch];
  return k.w00 * q00 + k.w10 * q10 + k.w01 * q01 + k.w11 * q11;
}

// SEL: channel-selective dword loads (else float4 loads as production); NC > 0: the normal stage
// unrolled over exactly NC cascades (all its loads issued together), else a runtime loop
// INC: the vertex's (i, j) advanced by the grid stride's (di, dj) with a carry instead of a 64-bit
// division and remainder per vertex
template <bool SEL, int NC, bool INC = false>
__global__ __launch_bounds__(256) void k_surface_v(SurfaceParams p, SurfacePlane plane, int64_t count,
                                                   float4* __restrict__ out)
{
#pragma clang fp contract(off)
  float tx = 0.0f, tz = 0.0f, cam_y = 0.0f;
  {
    const float fl = sqrtf(plane.fwd_x * plane.fwd_x + plane.fwd_z * plane.fwd_z);
    const float tx0 = plane.fwd_x / fl, tz0 = plane.fwd_z / fl;
    tx = (tx0 - tz0) * 0.70711f;
    tz = (tx0 + tz0) * 0.70711f;
    cam_y = fmaxf(plane.cam_y, 10.0f);
  }
  const int ncas = NC > 0 ? NC : p.count;
  const int side = plane.res + 1;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t idx0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int di = (int)(stride % side), dj = (int)(stride / side);
  int ic = (int)(idx0 % side), jc = (int)(idx0 / side);
  for (int64_t idx = idx0; idx < count; idx += stride)
  {
    int i, j;
    if constexpr (INC)
    {
      i = ic;
      j = jc;
      ic += di;
      jc += dj;
      if (ic >= side)
      {
        ic -= side;
        jc++;
      }
    }
    else
    {
      i = (int)(idx % side);
      j = (int)(idx / side);
    }
    const float x = -20.0f + 40.0f * (float)i / (float)plane.res + 15.0f;
    const float z = -20.0f + 40.0f * (float)j / (float)plane.res + 15.0f;
    float rx = tx * x - tz * z, rz = x * tz + z * tx;
    const float len0 = sqrtf(rx * rx + rz * rz);
    const float kk = powf(fmaxf(len0, 1.0f), 1.2f) * cam_y * 0.04f;
    float px = rx * kk + plane.cam_x;
    float pz = rz * kk + plane.cam_z;
    float py = 0.0f;
    for (int c = 0; c < ncas; c++)
    {
      const float u = px / p.c[c].plane, v = pz / p.c[c].plane;
      const Taps k = taps_of(p.n, u, v);
      const float* hm = reinterpret_cast<const float*>(p.c[c].height);
      const float* dm = reinterpret_cast<const float*>(p.c[c].disp);
      float h0, h3, d0;
      if constexpr (SEL)
      {
        h0 = tap_sum<4>(hm, k, 0);
        h3 = tap_sum<4>(hm, k, 3);
        d0 = tap_sum<4>(dm, k, 0);
      }
      else
      {
        float d1[4], d2[4];
        sample_linear_repeat<4>(hm, p.n, u, v, d1);
        sample_linear_repeat<4>(dm, p.n, u, v, d2);
        h0 = d1[0];
        h3 = d1[3];
        d0 = d2[0];
      }
      px += p.c[c].scale * h3;
      py += h0;
      pz += p.c[c].scale * d0;
    }
    float d[4] = {0.0f, 0.0f, 0.0f, 0.0f}, jac = 0.0f;
    auto normal_stage = [&](int c) __attribute__((always_inline)) {
      const float u = px / p.c[c].plane, v = pz / p.c[c].plane;
      const float* hm = reinterpret_cast<const float*>(p.c[c].height);
      const float* dm = reinterpret_cast<const float*>(p.c[c].disp);
      float h1, h2, e1, e2, jj;
      if constexpr (SEL)
      {
        const Taps k = taps_of(p.n, u, v);
        h1 = tap_sum<4>(hm, k, 1);
        h2 = tap_sum<4>(hm, k, 2);
        e1 = tap_sum<4>(dm, k, 1);
        e2 = tap_sum<4>(dm, k, 2);
        jj = tap_sum<1>(p.c[c].jac, k, 0);
      }
      else
      {
        float d1[4], d2[4];
        sample_linear_repeat<4>(hm, p.n, u, v, d1);
        sample_linear_repeat<4>(dm, p.n, u, v, d2);
        sample_linear_repeat<1>(p.c[c].jac, p.n, u, v, &jj);
        h1 = d1[1];
        h2 = d1[2];
        e1 = d2[1];
        e2 = d2[2];
      }
      jac += jj / (float)ncas;
      const float f = p.c[c].scale;
      d[0] += h1;
      d[1] += e1 * f;
      d[2] += h2;
      d[3] += e2 * f;
    };
    if constexpr (NC > 0)
    {
#pragma unroll
      for (int c = 0; c < NC; c++)
        normal_stage(c);
    }
    else
      for (int c = 0; c < ncas; c++)
        normal_stage(c);
    const float sx = d[0] / (1.0f + d[1]), sz = d[2] / (1.0f + d[3]);
    const float nx = -sx, ny = 1.0f, nz = -sz;
    const float len = sqrtf(nx * nx + ny * ny + nz * nz);
    out[2 * idx] = make_float4(px, py, pz, jac);
    out[2 * idx + 1] = make_float4(nx / len, ny / len, nz / len, 0.0f);
  }
}


// ATLAS: per cascade two repacked maps, a[texel] = (h, Dx, Dz, 0) for the vertex stage and
// b[texel] = (dh/dx, dh/dz, dDx/dx, dDz/dz) + jac[texel] for the normal stage: one 16-B load per tap
// and stage (plus the Jacobian's dword) instead of one dword per channel
struct Atlas
{
  const float4* a[3];
  const float4* b[3];
};

__global__ void k_atlas(SurfaceParams p, float4* a0, float4* b0)
{
  const int nn = p.n * p.n;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < p.count * nn; idx += gridDim.x * blockDim.x)
  {
    const int c = idx / nn, t = idx - c * nn;
    const float4 h = p.c[c].height[t], d = p.c[c].disp[t];
    a0[idx] = make_float4(h.x, h.w, d.x, 0.0f);
    b0[idx] = make_float4(h.y, h.z, d.y, d.z);
  }
}

__global__ __launch_bounds__(256) void k_surface_atlas(SurfaceParams p, Atlas at, SurfacePlane plane, int64_t count,
                                                       float4* __restrict__ out)
{
#pragma clang fp contract(off)
  float tx = 0.0f, tz = 0.0f, cam_y = 0.0f;
  {
    const float fl = sqrtf(plane.fwd_x * plane.fwd_x + plane.fwd_z * plane.fwd_z);
    const float tx0 = plane.fwd_x / fl, tz0 = plane.fwd_z / fl;
    tx = (tx0 - tz0) * 0.70711f;
    tz = (tx0 + tz0) * 0.70711f;
    cam_y = fmaxf(plane.cam_y, 10.0f);
  }
  const int ncas = p.count;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < count; idx += (int64_t)gridDim.x * blockDim.x)
  {
    const int side = plane.res + 1;
    const int i = (int)(idx % side), j = (int)(idx / side);
    const float x = -20.0f + 40.0f * (float)i / (float)plane.res + 15.0f;
    const float z = -20.0f + 40.0f * (float)j / (float)plane.res + 15.0f;
    float rx = tx * x - tz * z, rz = x * tz + z * tx;
    const float len0 = sqrtf(rx * rx + rz * rz);
    const float kk = powf(fmaxf(len0, 1.0f), 1.2f) * cam_y * 0.04f;
    float px = rx * kk + plane.cam_x;
    float pz = rz * kk + plane.cam_z;
    float py = 0.0f;
    for (int c = 0; c < ncas; c++)
    {
      const float u = px / p.c[c].plane, v = pz / p.c[c].plane;
      const Taps k = taps_of(p.n, u, v);
      const float4 q00 = at.a[c][k.o00], q10 = at.a[c][k.o10], q01 = at.a[c][k.o01], q11 = at.a[c][k.o11];
      const float h0 = k.w00 * q00.x + k.w10 * q10.x + k.w01 * q01.x + k.w11 * q11.x;
      const float h3 = k.w00 * q00.y + k.w10 * q10.y + k.w01 * q01.y + k.w11 * q11.y;
      const float d0 = k.w00 * q00.z + k.w10 * q10.z + k.w01 * q01.z + k.w11 * q11.z;
      px += p.c[c].scale * h3;
      py += h0;
      pz += p.c[c].scale * d0;
    }
    float d[4] = {0.0f, 0.0f, 0.0f, 0.0f}, jac = 0.0f;
    for (int c = 0; c < ncas; c++)
    {
      const float u = px / p.c[c].plane, v = pz / p.c[c].plane;
      const Taps k = taps_of(p.n, u, v);
      const float4 q00 = at.b[c][k.o00], q10 = at.b[c][k.o10], q01 = at.b[c][k.o01], q11 = at.b[c][k.o11];
      jac += tap_sum<1>(p.c[c].jac, k, 0) / (float)ncas;
      const float f = p.c[c].scale;
      d[0] += k.w00 * q00.x + k.w10 * q10.x + k.w01 * q01.x + k.w11 * q11.x;
      d[1] += (k.w00 * q00.z + k.w10 * q10.z + k.w01 * q01.z + k.w11 * q11.z) * f;
      d[2] += k.w00 * q00.y + k.w10 * q10.y + k.w01 * q01.y + k.w11 * q11.y;
      d[3] += (k.w00 * q00.w + k.w10 * q10.w + k.w01 * q01.w + k.w11 * q11.w) * f;
    }
    const float sx = d[0] / (1.0f + d[1]), sz = d[2] / (1.0f + d[3]);
    const float nx = -sx, ny = 1.0f, nz = -sz;
    const float len = sqrtf(nx * nx + ny * ny + nz * nz);
    out[2 * idx] = make_float4(px, py, pz, jac);
    out[2 * idx + 1] = make_float4(nx / len, ny / len, nz / len, 0.0f);
  }
}

__global__ void fill_maps(float* p, size_t n, unsigned seed, float amp)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
  {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    p[i] = amp * (((float)(h & 0xffff) - 32768.0f) * (1.0f / 32768.0f));
  }
}

template <typename F>
float time_ms(F&& launch, int reps)
{
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  CHECK(launch());
  CHECK(hipDeviceSynchronize());
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

}  // namespace

int main()
{
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  constexpr int n = 256, C = 3;
  const float planes[C] = {5.0f, 17.0f, 101.0f};
  SurfaceParams p{};
  p.count = C;
  p.n = n;
  for (int c = 0; c < C; c++)
  {
    float4 *h, *d;
    float* j;
    CHECK(hipMalloc(&h, (size_t)n * n * 16));
    CHECK(hipMalloc(&d, (size_t)n * n * 16));
    CHECK(hipMalloc(&j, (size_t)n * n * 4));
    hipLaunchKernelGGL(fill_maps, dim3(256), dim3(256), 0, 0, reinterpret_cast<float*>(h), (size_t)n * n * 4, 11u + c, 0.5f);
    hipLaunchKernelGGL(fill_maps, dim3(256), dim3(256), 0, 0, reinterpret_cast<float*>(d), (size_t)n * n * 4, 23u + c, 0.3f);
    hipLaunchKernelGGL(fill_maps, dim3(256), dim3(256), 0, 0, j, (size_t)n * n, 37u + c, 1.0f);
    p.c[c] = SurfaceCascade{h, d, j, planes[c], 1.0f};
  }
  float4 *atl_a, *atl_b;
  CHECK(hipMalloc(&atl_a, (size_t)C * n * n * 16));
  CHECK(hipMalloc(&atl_b, (size_t)C * n * n * 16));
  Atlas atl{};
  for (int c = 0; c < C; c++)
  {
    atl.a[c] = atl_a + (size_t)c * n * n;
    atl.b[c] = atl_b + (size_t)c * n * n;
  }
  for (int res : {1024, 4096})
  {
    const SurfacePlane plane{res, 3.0f, 5.0f, -2.0f, -0.6f, 0.8f};
    const int64_t pts = (int64_t)(res + 1) * (res + 1);
    float4 *o0, *o1;
    CHECK(hipMalloc(&o0, pts * 32));
    CHECK(hipMalloc(&o1, pts * 32));
    const long cap = (long)cus * 8;
    const long blocks = std::min<long>((pts + 255) / 256, cap);
    std::vector<std::string> names = {"production k_surface (dword channels)", "float4 loads (round-6 production before)",
                                      "dword channels, runtime loops", "dword channels, normal stage unrolled (3)",
                                      "dword channels, unrolled, grid x2", "dword channels, unrolled, grid x4",
                                      "dword channels, incremental (i, j)", "dword channels, incremental, grid x4",
                                      "atlas: repack + sample", "atlas: sample only"};
    std::vector<std::function<hipError_t()>> runs = {
        [&] { return launch_surface(p, plane, nullptr, pts, o0, 0, cus); },
        [&] {
          hipLaunchKernelGGL((k_surface_v<false, 0>), dim3(blocks), dim3(256), 0, 0, p, plane, pts, o1);
          return hipGetLastError();
        },
        [&] {
          hipLaunchKernelGGL((k_surface_v<true, 0>), dim3(blocks), dim3(256), 0, 0, p, plane, pts, o1);
          return hipGetLastError();
        },
        [&] {
          hipLaunchKernelGGL((k_surface_v<true, 3>), dim3(blocks), dim3(256), 0, 0, p, plane, pts, o1);
          return hipGetLastError();
        },
        [&] {
          const long b2 = std::min<long>((pts + 255) / 256, cap * 2);
          hipLaunchKernelGGL((k_surface_v<true, 3>), dim3(b2), dim3(256), 0, 0, p, plane, pts, o1);
          return hipGetLastError();
        },
        [&] {
          const long b4 = std::min<long>((pts + 255) / 256, cap * 4);
          hipLaunchKernelGGL((k_surface_v<true, 3>), dim3(b4), dim3(256), 0, 0, p, plane, pts, o1);
          return hipGetLastError();
        },
        [&] {
          hipLaunchKernelGGL((k_surface_v<true, 0, true>), dim3(blocks), dim3(256), 0, 0, p, plane, pts, o1);
          return hipGetLastError();
        },
        [&] {
          const long b4 = std::min<long>((pts + 255) / 256, cap * 4);
          hipLaunchKernelGGL((k_surface_v<true, 0, true>), dim3(b4), dim3(256), 0, 0, p, plane, pts, o1);
          return hipGetLastError();
        },
        [&] {
          hipLaunchKernelGGL(k_atlas, dim3(cus * 4), dim3(256), 0, 0, p, atl_a, atl_b);
          hipLaunchKernelGGL(k_surface_atlas, dim3(blocks), dim3(256), 0, 0, p, atl, plane, pts, o1);
          return hipGetLastError();
        },
        [&] {
          hipLaunchKernelGGL(k_surface_atlas, dim3(blocks), dim3(256), 0, 0, p, atl, plane, pts, o1);
          return hipGetLastError();
        }};
    std::vector<float> ref(pts * 8), got(pts * 8);
    CHECK(runs[0]());
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(ref.data(), o0, pts * 32, hipMemcpyDeviceToHost));
    for (size_t k = 1; k < runs.size(); k++)
    {
      CHECK(hipMemset(o1, 0xff, pts * 32));
      CHECK(runs[k]());
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemcpy(got.data(), o1, pts * 32, hipMemcpyDeviceToHost));
      std::printf("mesh %d: %s: %s\n", res, names[k].c_str(),
                  std::memcmp(ref.data(), got.data(), pts * 32) == 0 ? "bit-identical" : "DIFFERS");
    }
    std::vector<std::vector<float>> t(runs.size());
    for (int r = 0; r < 7; r++)
      for (size_t k = 0; k < runs.size(); k++)
        t[k].push_back(time_ms(runs[k], 10));
    for (size_t k = 0; k < runs.size(); k++)
    {
      std::sort(t[k].begin(), t[k].end());
      std::printf("mesh %4d (%9lld vertices) %-44s median %8.4f ms  %7.2f G vertices/s  %7.1f GB/s out\n", res,
                  (long long)pts, names[k].c_str(), t[k][3], pts / (t[k][3] * 1e6), 32.0 * pts / (t[k][3] * 1e6));
    }
    CHECK(hipFree(o0));
    CHECK(hipFree(o1));
  }
  return 0;
}
