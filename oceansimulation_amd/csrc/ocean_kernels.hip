// ocean_kernels.hip — gfx950 device code of the ocean hot path, core translation unit: h0 seeding
// (generateSpectrum), the debug Hash, the Nyquist-row term of the half-spectrum paths and the surface
// consumer, with their launchers and the host-side size helpers. The frame passes live in
// launch_half.hip (whole grids of 1024 .. 4096), launch_slab.hip (slabs, and 8192 / 16384) and
// launch_fft.hip (standalone EncodeIFFT and the full-spectrum path); their kernels in device/k_*.h.
//
// Reference semantics (paths relative to the reference root):
//   spectrum seeding      resources/spectrum.compute:38-172   (generateSpectrum)
//   evolve + packing      resources/spectrum.compute:183-240  (prepareFFT)
//   2D inverse FFT        resources/fft.compute:21-88 driven by src/FFTCalculator.cpp:73-114
//                         == N^2 * ifft2(ifftshift(X)) per complex lane, no normalisation
//   Jacobian / foam       resources/spectrum.compute:246-259
//
// MI355X design (DESIGN.md has the byte accounting): every frame pass streams HBM in >= 128-B pieces;
// each 1D transform is a self-sorting Stockham FFT held in VGPRs (device/fft.h: 16 points per thread,
// radix-16 stages, split-plane packed complex math, LDS only between stages); fftShift is folded into
// load indices and no bit-reversal pass exists; grids are one-shot on the whole device, persistent
// under a CU budget (launch_common.h), and every item loop exits on an item count.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "ocean_internal.h"
#include "launch_common.h"
#include "device/evolve.h"
#include "device/fft.h"
#include "device/grid.h"
#include "device/memory.h"
#include "device/spectrum.h"

namespace oceanfft
{

// generateSpectrum (spectrum.compute:157-172): texel = (h0(k), conj(h0(-k))), -k taken as N - i.
// Stored strip-blocked, h0[xb][y][blk] (blk texel columns per strip, see ColFirstCfg), so the
// column pass reads each strip as one contiguous run. The reference keeps this image private
// (src/Generator.h:86), so its layout is internal.
__global__ __launch_bounds__(256) void k_generate_spectrum(SpectrumConsts s, int n, int blk, int x0, int width,
                                                          float4* __restrict__ h0, int rows)
{
  // columns [x0, x0 + width) of rows [0, rows) of the N x N spectrum (a rank's column slab; width =
  // n for a whole grid; rows = 1: the row y = 0 a slab's Nyquist-row term needs, [x])
  const int64_t total = (int64_t)width * rows;
  const float dim = (float)n;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x)
  {
    // idx enumerates the blocked layout: b fastest, then y, then xb
    const int b = (int)(idx % blk);
    const int64_t rest = idx / blk;
    const int y = (int)(rest % rows), xb = (int)(rest / rows);
    const int x = x0 + xb * blk + b;
    float2 a = spectrum_amplitude(s, (float)x, (float)y);
    float2 c = spectrum_amplitude(s, dim - (float)x, dim - (float)y);
    h0[idx] = make_float4(a.x, a.y, c.x, -c.y);
  }
}

// Whole grid, one amplitude evaluation per texel: texel (x, y) needs h0 at (x, y) and at its
// partner (N-x, N-y), and the partner's texel needs the same two values swapped, so one thread
// evaluates both points and writes both texels. Points run over the lower half y < N/2; the
// texels no pair reaches (row N/2, which mirrors onto itself, and column 0 of the upper half,
// whose partner column N is off the grid) are tail items with two evaluations each (O(N)).
// Bit-identical to k_generate_spectrum: same evaluator, same float arguments.
// Index math in 32 bits with shifts (n, blk powers of two; pairs + tail < 2^31 up to n = 16384):
// the 64-bit divisions by runtime n / blk cost ~100 VALU per point.
__global__ __launch_bounds__(256) void k_generate_spectrum_pairs(SpectrumConsts s, int logn, int lblk,
                                                                float4* __restrict__ h0)
{
  const int n = 1 << logn, half = n >> 1, blk = 1 << lblk;
  const int pairs = n * half, total = pairs + n + (half - 1);
  const float dim = (float)n;
  auto at = [&](int x, int y) {
    return ((size_t)(((x >> lblk) << logn) + y) << lblk) + (x & (blk - 1));
  };
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x)
  {
    int x, y;
    bool mirror;
    if (idx < pairs)  // blocked order over the lower half: b fastest, then y, then xb
    {
      const int b = idx & (blk - 1);
      const int rest = idx >> lblk;
      y = rest & (half - 1);
      x = ((rest >> (logn - 1)) << lblk) + b;
      mirror = x > 0 && y > 0;
    }
    else if (idx < pairs + n)
    {
      x = idx - pairs;
      y = half;
      mirror = false;
    }
    else
    {
      x = 0;
      y = half + 1 + (idx - pairs - n);
      mirror = false;
    }
    const float2 a = spectrum_amplitude(s, (float)x, (float)y);
    const float2 c = spectrum_amplitude(s, dim - (float)x, dim - (float)y);
    h0[at(x, y)] = make_float4(a.x, a.y, c.x, -c.y);
    if (mirror)
      h0[at(n - x, n - y)] = make_float4(c.x, c.y, a.x, -a.y);
  }
}

// Debug entry for bit-exact Hash parity (spectrum.compute:109-117).
__global__ void k_hash(const uint32_t* __restrict__ xy, int count, uint32_t* __restrict__ raw,
                       float2* __restrict__ uv)
{
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count)
  {
    raw[i] = hash_raw(xy[2 * i], xy[2 * i + 1]);
    uv[i] = hash_uniform(xy[2 * i], xy[2 * i + 1]);
  }
}

// The Nyquist-row term: for u = -u' (0 < u' < N/2) the pass-2 rebuild s_F conj(G_F(q, u')) misses
// (-1)^q Delta_F(u'), Delta_F(u') = F(-N/2, -u') - s_F conj(F(-N/2, u')). Its lanes (the kx
// factors of pass 2 applied to Delta) form one row spectrum per image, spec[c][img][x] (zero
// outside 0 < x < N/2); pass 2 adds (-1)^q spec to the lanes it rebuilds at u < 0.
// h0row (slabs, whose h0 holds only their strips): the row y = 0 texels of every column, [c][x].
// copies / copy_stride: the strip-dealt path writes the term into every destination block of the
// exchange buffer, so each frame's row pass reads the term of its own frame (the pipeline keeps two
// frames in flight).
// seed (the fused re-seed frame, h0 not materialised): the two row-0 texels are evaluated here.
// dst (the one-sided exchange): copy k goes to dst[k] + dst_off, this rank's block in rank k's
// receive slot, instead of spec + k * copy_stride.
__global__ __launch_bounds__(256) void k_half_nyquist(FrameParams fp, int n, int blk, const float4* __restrict__ h0,
                                                      float4* __restrict__ spec, const float4* __restrict__ h0row,
                                                      int copies, size_t copy_stride,
                                                      const SpectrumConsts* __restrict__ seed,
                                                      const uint64_t* __restrict__ dst, size_t dst_off)
{
  const int total = fp.cascades * n;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x)
    half_nyquist_texel(fp, n, blk, h0, spec, h0row, copies, copy_stride, seed, dst, dst_off, idx);
}

// ------------------------------------------------------------------------------------------------
// Frame signals of the one-sided slab exchange (ocean_peers, include/oceanfft.h). Every rank owns a
// small array of 32-bit flag words in uncached device memory; word `ready + q` counts the frames
// whose blocks rank q has stored into this rank's receive slots, word `freed + q` the frames whose
// receive slot rank q's row pass has finished reading. Peers write them through their IPC mappings
// (xGMI), this rank's own words locally. Values are frame numbers + 1, so they only grow.
// ------------------------------------------------------------------------------------------------
// k_peer_signal: one wave; lane q < ranks stores `value` into word `word` of rank q's flags with a
// system-scope release (the "freed" signal: the row pass before it in the stream only read).
__global__ __launch_bounds__(64) void k_peer_signal(uint32_t* const* __restrict__ flags, int ranks, int word,
                                                    uint32_t value)
{
  const int q = threadIdx.x;
  if (q < ranks)
    __hip_atomic_store(flags[q] + word, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// k_peer_signal_release: the "ready" signal after the puts. The put kernels' stores to the peers may
// still sit in the XCD L2s (each XCD has its own); kPeerReleaseBlocks workgroups, dealt over all 8
// XCDs, each write back their XCD's L2 (a system-scope release fence), then count themselves in on
// `counter` (this rank's flag memory); the last one in raises the flags, as k_peer_signal does.
// The counter only grows: the last workgroup of a launch is the one that sees a multiple of the
// block count minus one, so no reset is needed between frames.
constexpr int kPeerReleaseBlocks = 64;

__global__ __launch_bounds__(64) void k_peer_signal_release(uint32_t* const* __restrict__ flags, int ranks, int word,
                                                            uint32_t value, uint32_t* __restrict__ counter)
{
  if (threadIdx.x != 0)
    return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  const uint32_t n = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
  if ((n + 1) % kPeerReleaseBlocks != 0)
    return;
  for (int q = 0; q < ranks; q++)
    __hip_atomic_store(flags[q] + word, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// k_peer_wait: kPeerReleaseBlocks one-wave workgroups, dealt over the 8 XCDs like the release's; in
// each, lane q < ranks polls word `word0 + q` of this rank's flags until it reaches `target` (as a
// wrapping difference), then the wave runs a system-scope acquire fence. The acquire is symmetric to
// the release (round 6): every XCD's L2 drops its clean copies of peer-written
// lines (a slot the row pass of frame f - 2 read on all XCDs) from a wave running on that XCD, before
// the row pass (the next launch on the stream, whose own kernel-start acquire also invalidates the
// L1s and L2s) reads the slot; DESIGN.md §6 "Visibility". Every lane exits: on success, or when the
// wall clock passes `deadline_ticks` after the start, in which case err[0] records the word range that
// timed out (word0 + 1) and the frame goes on with whatever the slots hold; err stays set until
// ocean_peers_synchronize reports it (the waits of later frames return at once), and the peers then
// refuse new frames. A wait can never hold the GPU past its deadline.
__global__ __launch_bounds__(64) void k_peer_wait(const uint32_t* __restrict__ flags, int word0, int ranks,
                                                  uint32_t target, long long deadline_ticks, uint32_t* __restrict__ err)
{
  const int q = threadIdx.x;
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0)
    return;
  const long long t0 = wall_clock64();
  bool ok = q >= ranks;
  for (;;)
  {
    if (!ok)
      ok = (int)(__hip_atomic_load(flags + word0 + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - target) >= 0;
    if (__all(ok))
      break;
    if (wall_clock64() - t0 > deadline_ticks)
    {
      if (q == 0)
        __hip_atomic_store(err, (uint32_t)(word0 + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

hipError_t launch_peer_signal(uint32_t* const* flags, int ranks, int word, uint32_t value, hipStream_t stream)
{
  hipLaunchKernelGGL(k_peer_signal, dim3(1), dim3(64), 0, stream, flags, ranks, word, value);
  return hipGetLastError();
}

hipError_t launch_peer_signal_release(uint32_t* const* flags, int ranks, int word, uint32_t value, uint32_t* counter,
                                      hipStream_t stream)
{
  hipLaunchKernelGGL(k_peer_signal_release, dim3(kPeerReleaseBlocks), dim3(64), 0, stream, flags, ranks, word, value,
                     counter);
  return hipGetLastError();
}

hipError_t launch_peer_wait(const PeerWait& w, hipStream_t stream)
{
  hipLaunchKernelGGL(k_peer_wait, dim3(kPeerReleaseBlocks), dim3(64), 0, stream, w.flags, w.word0, w.ranks, w.target,
                     w.deadline_ticks, w.err);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Surface consumer: resources/waveShader.glsl evaluated per mesh vertex on the
// generator's maps. Vertex stage (:101-110): each cascade samples heightMap/displacementMap at
// pos.xz / planeSize, the position the earlier cascades already displaced, and adds
// (scale * Dx, h, scale * Dz). Fragment stage at the displaced position (:127-144): summed slopes
// -> normal, averaged Jacobian. Sampling is GL_LINEAR + GL_REPEAT (src/Generator.cpp:116-119) in
// fp32 with the specification's weights, unfused and with correctly rounded division / sqrt, so
// the oracle restatement (oracle_surface_vertex) is matched bit for bit. Memory: the maps of a
// scene (3 x 256^2 x 36 B) live in L2; per vertex 32 B are written.
// ------------------------------------------------------------------------------------------------
// The four taps and weights of one sample: the texel indices of (i0, j0), (i1, j0), (i0, j1), (i1, j1).
struct LinearTaps
{
  int o00, o10, o01, o11;
  float w00, w10, w01, w11;
};

__device__ __forceinline__ LinearTaps linear_repeat_taps(int n, float u, float v)
{
#pragma clang fp contract(off)
  const float s = u * (float)n - 0.5f, t = v * (float)n - 0.5f;
  const float fs = floorf(s), ft = floorf(t);
  const float a = s - fs, b = t - ft;
  const int m = n - 1;  // n is a power of two: & m is the repeat wrap, also for negative indices
  const int i0 = (int)fs & m, j0 = (int)ft & m, i1 = (i0 + 1) & m, j1 = (j0 + 1) & m;
  return LinearTaps{j0 * n + i0, j0 * n + i1, j1 * n + i0, j1 * n + i1, (1.0f - a) * (1.0f - b), a * (1.0f - b),
                    (1.0f - a) * b, a * b};
}

// Channel ch of a map of CH floats per texel, filtered: each stage loads only the channels it uses, one
// dword per tap (the vertex stage 3 of 8, the normal stage 5 of 9): 2.95 -> 2.49 ms for the 4096^2-quad
// mesh, bit-identical (tools/microbench/surfbench, profiles/r06_surfbench.log). A sampling wave's taps
// are scattered (the camera warp spreads far vertices ~10 texels apart on a 5 m cascade), so the cost
// is per load instruction: ATLAS repacks the channels each stage uses into one 16-B texel (one load per
// tap and stage, plus the Jacobian's dword): 2.47 -> 1.35 ms with the repack included, 0.212 -> 0.121 ms
// for the 1024^2-quad mesh, bit-identical (profiles/r06_surfbench2.log).
template <int CH>
__device__ __forceinline__ float linear_channel(const float* __restrict__ tex, const LinearTaps& k, int ch)
{
#pragma clang fp contract(off)
  const float q00 = tex[k.o00 * CH + ch], q10 = tex[k.o10 * CH + ch], q01 = tex[k.o01 * CH + ch],
              q11 = tex[k.o11 * CH + ch];
  return k.w00 * q00 + k.w10 * q10 + k.w01 * q01 + k.w11 * q11;
}

// The bilinear sum of the four taps' lanes x, y, z, w (each as linear_channel's sum)
__device__ __forceinline__ float4 linear_texel(const float4* __restrict__ tex, const LinearTaps& k)
{
#pragma clang fp contract(off)
  const float4 q00 = tex[k.o00], q10 = tex[k.o10], q01 = tex[k.o01], q11 = tex[k.o11];
  return make_float4(k.w00 * q00.x + k.w10 * q10.x + k.w01 * q01.x + k.w11 * q11.x,
                     k.w00 * q00.y + k.w10 * q10.y + k.w01 * q01.y + k.w11 * q11.y,
                     k.w00 * q00.z + k.w10 * q10.z + k.w01 * q01.z + k.w11 * q11.z,
                     k.w00 * q00.w + k.w10 * q10.w + k.w01 * q01.w + k.w11 * q11.w);
}

// the surface atlas of the cascades' maps (SurfaceParams::atlas)
__global__ __launch_bounds__(256) void k_surface_atlas(SurfaceParams p)
{
  const int nn = p.n * p.n;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < p.count * nn; idx += gridDim.x * blockDim.x)
  {
    const int c = idx / nn, t = idx - c * nn;
    const float4 h = p.c[c].height[t], d = p.c[c].disp[t];
    p.atlas[(size_t)(2 * c) * nn + t] = make_float4(h.x, h.w, d.x, 0.0f);
    p.atlas[(size_t)(2 * c + 1) * nn + t] = make_float4(h.y, h.z, d.y, d.z);
  }
}

template <bool ATLAS>
__global__ __launch_bounds__(256) void k_surface(SurfaceParams p, SurfacePlane plane, const float2* __restrict__ xz,
                                                 int64_t count, float4* __restrict__ out)
{
#pragma clang fp contract(off)
  float tx = 0.0f, tz = 0.0f, cam_y = 0.0f;
  if (plane.res > 0)
  {
    // turnDir = normalize(forward.xz) rotated by 45 degrees (waveShader.glsl:84-88)
    const float fl = sqrtf(plane.fwd_x * plane.fwd_x + plane.fwd_z * plane.fwd_z);
    const float tx0 = plane.fwd_x / fl, tz0 = plane.fwd_z / fl;
    tx = (tx0 - tz0) * 0.70711f;
    tz = (tx0 + tz0) * 0.70711f;
    cam_y = fmaxf(plane.cam_y, 10.0f);
  }
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < count;
       idx += (int64_t)gridDim.x * blockDim.x)
  {
    float px, pz;
    if (plane.res > 0)
    {
      // plane vertex (src/Renderer.cpp:18), + (15, 0, 15), rotate, distance scale, camera offset
      const int side = plane.res + 1;
      const int i = (int)(idx % side), j = (int)(idx / side);
      const float x = -20.0f + 40.0f * (float)i / (float)plane.res + 15.0f;
      const float z = -20.0f + 40.0f * (float)j / (float)plane.res + 15.0f;
      float rx = tx * x - tz * z, rz = x * tz + z * tx;
      const float len = sqrtf(rx * rx + rz * rz);
      const float k = powf(fmaxf(len, 1.0f), 1.2f) * cam_y * 0.04f;
      px = rx * k + plane.cam_x;
      pz = rz * k + plane.cam_z;
    }
    else
    {
      const float2 q = xz[idx];
      px = q.x;
      pz = q.y;
    }
    float py = 0.0f;
    const int nn = p.n * p.n;
    for (int c = 0; c < p.count; c++)
    {
      const float u = px / p.c[c].plane, v = pz / p.c[c].plane;
      const LinearTaps k = linear_repeat_taps(p.n, u, v);
      float h, dx, dz;
      if constexpr (ATLAS)
      {
        const float4 a = linear_texel(p.atlas + (size_t)(2 * c) * nn, k);
        h = a.x;
        dx = a.y;
        dz = a.z;
      }
      else
      {
        const float* hm = reinterpret_cast<const float*>(p.c[c].height);
        const float* dm = reinterpret_cast<const float*>(p.c[c].disp);
        h = linear_channel<4>(hm, k, 0);
        dx = linear_channel<4>(hm, k, 3);
        dz = linear_channel<4>(dm, k, 0);
      }
      px += p.c[c].scale * dx;
      py += h;
      pz += p.c[c].scale * dz;
    }
    float d[4] = {0.0f, 0.0f, 0.0f, 0.0f}, jac = 0.0f;
    for (int c = 0; c < p.count; c++)
    {
      const float u = px / p.c[c].plane, v = pz / p.c[c].plane;
      const LinearTaps k = linear_repeat_taps(p.n, u, v);
      float hx, dxx, hz, dzz;
      if constexpr (ATLAS)
      {
        const float4 b = linear_texel(p.atlas + (size_t)(2 * c + 1) * nn, k);
        hx = b.x;
        hz = b.y;
        dxx = b.z;
        dzz = b.w;
      }
      else
      {
        const float* hm = reinterpret_cast<const float*>(p.c[c].height);
        const float* dm = reinterpret_cast<const float*>(p.c[c].disp);
        hx = linear_channel<4>(hm, k, 1);
        dxx = linear_channel<4>(dm, k, 1);
        hz = linear_channel<4>(hm, k, 2);
        dzz = linear_channel<4>(dm, k, 2);
      }
      jac += linear_channel<1>(p.c[c].jac, k, 0) / (float)p.count;
      const float f = p.c[c].scale;
      d[0] += hx;        // dh/dx
      d[1] += dxx * f;   // dDx/dx
      d[2] += hz;        // dh/dz
      d[3] += dzz * f;   // dDz/dz
    }
    const float sx = d[0] / (1.0f + d[1]), sz = d[2] / (1.0f + d[3]);
    const float nx = -sx, ny = 1.0f, nz = -sz;
    const float len = sqrtf(nx * nx + ny * ny + nz * nz);
    out[2 * idx] = make_float4(px, py, pz, jac);
    out[2 * idx + 1] = make_float4(nx / len, ny / len, nz / len, 0.0f);
  }
}

// ------------------------------------------------------------------------------------------------
// Host-side launchers and size helpers.
// ------------------------------------------------------------------------------------------------
size_t seed_consts_bytes() { return sizeof(SpectrumConsts); }

void seed_consts(const OceanSettings& s, int n, void* out) { *static_cast<SpectrumConsts*>(out) = spectrum_consts(s, n); }

int spectrum_block(int logn)
{
  int t = 1 << (logn - 4);
  return t >= 1024 ? 1 : (t >= 512 ? 2 : (t < 4 ? t : 4));
}

hipError_t launch_generate_spectrum(const OceanSettings& s, int n, float4* h0, hipStream_t stream, int cus, int x0,
                                    int width, int blk)
{
  int logn = 0;
  while ((1 << logn) < n)
    logn++;
  if (width <= 0)
    width = n;
  if (blk <= 0)
    blk = spectrum_block(logn);
  const bool whole = x0 == 0 && width == n;  // a slab's partner columns belong to other ranks
  long total = whole ? (long)n * (n / 2) + n + n / 2 - 1 : (long)n * width;
  long blocks = (total + 255) / 256;
  long cap = (long)cus * 16;
  if (blocks > cap)
    blocks = cap;
  if (whole)
  {
    int lblk = 0;
    while ((1 << lblk) < blk)
      lblk++;
    hipLaunchKernelGGL(k_generate_spectrum_pairs, dim3((unsigned)blocks), dim3(256), 0, stream,
                       spectrum_consts(s, n), logn, lblk, h0);
  }
  else
    hipLaunchKernelGGL(k_generate_spectrum, dim3((unsigned)blocks), dim3(256), 0, stream, spectrum_consts(s, n), n,
                       blk, x0, width, h0, n);
  return hipGetLastError();
}

hipError_t launch_surface(const SurfaceParams& p, const SurfacePlane& plane, const float2* xz, int64_t count,
                          float4* out, hipStream_t stream, int cus)
{
  if (count <= 0)
    return hipSuccess;
  long blocks = (long)((count + 255) / 256);
  const long cap = (long)cus * 8;
  if (blocks > cap)
    blocks = cap;
  if (p.atlas)
  {
    const long texels = (long)p.count * p.n * p.n;
    long ab = (texels + 255) / 256;
    if (ab > (long)cus * 4)
      ab = (long)cus * 4;
    hipLaunchKernelGGL(k_surface_atlas, dim3((unsigned)ab), dim3(256), 0, stream, p);
    hipLaunchKernelGGL(k_surface<true>, dim3((unsigned)blocks), dim3(256), 0, stream, p, plane, xz, count, out);
  }
  else
    hipLaunchKernelGGL(k_surface<false>, dim3((unsigned)blocks), dim3(256), 0, stream, p, plane, xz, count, out);
  return hipGetLastError();
}

size_t surface_atlas_texels(const SurfaceParams& p) { return (size_t)2 * p.count * p.n * p.n; }

// The repack reads 36 B and writes 32 B per map texel and launches one more kernel; sampling from the
// atlas saves ~90 ps per vertex (profiles/r06_surfbench2.log). Used when the request's vertices
// outnumber the maps' texels 4 : 1 (and are at least 64 Ki) and the atlas stays within 256 MiB.
bool surface_use_atlas(const SurfaceParams& p, int64_t points)
{
  const size_t texels = surface_atlas_texels(p);
  return points >= 65536 && (uint64_t)points >= 2 * (uint64_t)texels && texels * 16 <= ((size_t)256 << 20);
}

// A plain 16-B copy on a fixed number of 256-thread workgroups (ocean_debug_copy): bench.py paces the
// one-GPU emulation of a slab rank's exchange traffic with it (the workgroup count sets the rate).
__global__ __launch_bounds__(256) void k_debug_copy(const float4* __restrict__ src, float4* __restrict__ dst, size_t n16)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

hipError_t launch_debug_copy(void* dst, const void* src, size_t bytes, int workgroups, hipStream_t stream)
{
  hipLaunchKernelGGL(k_debug_copy, dim3(workgroups), dim3(256), 0, stream, static_cast<const float4*>(src),
                     static_cast<float4*>(dst), bytes / 16);
  return hipGetLastError();
}

hipError_t launch_hash(const uint32_t* xy, int count, uint32_t* raw, float2* uv, hipStream_t stream)
{
  hipLaunchKernelGGL(k_hash, dim3((count + 255) / 256), dim3(256), 0, stream, xy, count, raw, uv);
  return hipGetLastError();
}

hipError_t launch_generate_spectrum_row(const OceanSettings& s, int n, float4* row, hipStream_t stream)
{
  // the slab kernel over one row: the same evaluator in the same code, so bit-identical texels
  hipLaunchKernelGGL(k_generate_spectrum, dim3((n + 255) / 256), dim3(256), 0, stream, spectrum_consts(s, n), n, 1, 0,
                     n, row, 1);
  return hipGetLastError();
}


hipError_t launch_half_nyquist(const FrameParams& fp, int n, int blk, const float4* h0, float4* spec, const float4* h0row,
                               int copies, size_t copy_stride, const void* seed, hipStream_t stream, int cus,
                               const uint64_t* dst, size_t dst_off)
{
  long blocks = ((long)fp.cascades * n + 255) / 256;
  if (blocks > (long)cus * 4)
    blocks = (long)cus * 4;
  hipLaunchKernelGGL(k_half_nyquist, dim3((unsigned)blocks), dim3(256), 0, stream, fp, n, blk, h0, spec, h0row, copies,
                     copy_stride, static_cast<const SpectrumConsts*>(seed), dst, dst_off);
  return hipGetLastError();
}

// The largest H-retention that compiles without spills for this size (see k_cols_evolve).
int default_keep(int logn) { return logn >= 13 ? 0 : (logn == 12 ? 4 : 16); }

bool rows_need_transpose(int logn) { return spectrum_block(logn) == 1 && (1 << logn) >= 64; }

template <int LOGN>
static int slab_min_width_impl()
{
  using K = ColFirstCfg<LOGN>;
  int m = K::C1 > K::RPW2 ? K::C1 : K::RPW2;
  if (rows_need_transpose(LOGN))
    m = m > 64 ? m : 64;
  return m;
}

int slab_min_width(int logn)
{
  switch (logn)
  {
  case 4: return slab_min_width_impl<4>();
  case 5: return slab_min_width_impl<5>();
  case 6: return slab_min_width_impl<6>();
  case 7: return slab_min_width_impl<7>();
  case 8: return slab_min_width_impl<8>();
  case 9: return slab_min_width_impl<9>();
  case 10: return slab_min_width_impl<10>();
  case 11: return slab_min_width_impl<11>();
  case 12: return slab_min_width_impl<12>();
  case 13: return slab_min_width_impl<13>();
  case 14: return slab_min_width_impl<14>();
  default: return 1 << 30;
  }
}

bool fourstep_table(int logn) { return logn == 13 || logn == 14; }

int twiddle_entries(int logn)
{
  int lb = logn / 2;
  return (1 << lb) + (1 << (logn - lb));
}

}  // namespace oceanfft
