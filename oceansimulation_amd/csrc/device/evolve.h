// device/evolve.h — per-frame evolution h(k,t) and packing of the two RGBA32F images
// (resources/spectrum.compute:183-240).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device/spectrum.h"
#include "device/fft.h"

namespace oceanfft
{

// ------------------------------------------------------------------------------------------------
// Evolution + packing, resources/spectrum.compute:183-240.
// ------------------------------------------------------------------------------------------------
struct KVec
{
  float kx, kz, dirx, dirz, k;
  float inv;  // 1/|k| (0 at k = 0)
};

// Correctly rounded sqrt for the normal-range, non-negative arguments of the evolution (|k|^2 >=
// dk^2 ~ 1e-6; 0 maps to 0): hardware v_sqrt_f32 (<= 1 ulp) plus one residual test per neighbour,
// 9 VALU instead of hipcc's ~15 with denormal scaling. |k| and w must be bit-identical to the
// oracle's: the phase w*t multiplies any ulp of w by t (1e2-1e4 s of simulated time).
__device__ __forceinline__ float sqrt_rn(float x)
{
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __int_as_float(__float_as_int(s) - 1), sp = __int_as_float(__float_as_int(s) + 1);
  float r = s;
  if (fmaf(-sm, s, x) <= 0.0f)
    r = sm;
  if (fmaf(-sp, s, x) > 0.0f)
    r = sp;
  return r;
}

__device__ __forceinline__ KVec make_kvec(int x, int y, float dim, float dk)
{
#pragma clang fp contract(off)  // the reference's unfused float expression order
  KVec r;
  r.kx = ((float)x - dim / 2.0f) * dk;
  r.kz = ((float)y - dim / 2.0f) * dk;
  // |k| (spectrum.compute:189-192) correctly rounded, since it feeds the phase; normalize(kVec)
  // only scales the choppy terms and uses the hardware v_rsq_f32 (<= 1 ulp) instead of a
  // correctly rounded division (~10 VALU).
  const float len2 = r.kx * r.kx + r.kz * r.kz;
  const float inv = len2 == 0.0f ? 0.0f : __builtin_amdgcn_rsqf(len2);
  r.inv = inv;
  r.dirx = r.kx * inv;
  r.dirz = r.kz * inv;
  r.k = sqrt_rn(len2) + 1e-6f;
  return r;
}

// Dispersion (spectrum.compute:38-44) for the per-frame evolution. Same formula; tanh(kh), needed
// only when kh < 2*pi (very long waves), is evaluated as an odd series for kh < 1/8 (|err| < 1e-10)
// and as 1 - 2/(1 + e^{2kh}) above — a few VGPRs instead of ocml tanhf's.
__device__ __forceinline__ float dispersion_evolve(float k, float g, float h)
{
#pragma clang fp contract(off)  // bit-identical w in the deep-water case (tanh = 1)
  const float kh = k * h;
  float t = 1.0f;
  if (kh < 2.0f * OCEAN_PI)
  {
    const float x2 = kh * kh;
    t = kh < 0.125f ? kh * fmaf(fmaf(fmaf(-17.0f / 315.0f, x2, 2.0f / 15.0f), x2, -1.0f / 3.0f), x2, 1.0f)
                    : 1.0f - 2.0f / (1.0f + expf(2.0f * kh));
  }
  const float omegaSquared = (g * k + kSigmaSurface / kRhoWater * k * k * k) * t;
  return sqrt_rn(omegaSquared);
}

// sin/cos of a large fp32 phase (w*t reaches 1e3-1e7 rad). The phase is reduced to a fraction of a
// revolution in double (exact to ~1e-16 rev for |x| < 1e7) and fed to the hardware v_sin_f32 /
// v_cos_f32, which take revolutions (absolute error ~3e-7, the class of the reference shader's own
// GLSL sin/cos). ~10 VALU slots instead of ~35 for a polynomial kernel with quadrant logic, and no
// Payne-Hanek slow path (ocml's sincosf costs ~60 VGPRs that a 1024-thread workgroup lacks).
__device__ __forceinline__ void sincos_phase(float x, float* s, float* c)
{
  const double rev = (double)x * 0.15915494309189533577;  // 1 / (2 pi)
  const float f = (float)(rev - rint(rev));                // [-1/2, 1/2] revolution
  *s = __builtin_amdgcn_sinf(f);
  *c = __builtin_amdgcn_cosf(f);
}

// heightAmp = h0 * e^{i w t} + conj-partner * e^{-i w t}
__device__ __forceinline__ float2 evolve(float4 a, float k, const CascadeFrame& f)
{
#pragma clang fp contract(off)  // rounds identically wherever it is inlined (rolled or unrolled loops)
#ifdef OCEAN_ABLATE_EVOLVE  // timing ablation (tools/microbench): no dispersion / sin / cos, wrong results
  float ws = k * f.time, wc = k;
#else
  float phase = dispersion_evolve(k, f.g, f.h) * f.time;
  float ws, wc;
  sincos_phase(phase, &ws, &wc);
#endif
  float ampx = a.x * wc - a.y * ws;
  float ampy = a.x * ws + a.y * wc;
  float ws2 = -ws;
  float oppx = a.z * wc - a.w * ws2;
  float oppy = a.z * ws2 + a.w * wc;
  return make_float2(ampx + oppx, ampy + oppy);
}

// heightMap texel = (H + i*dH/dx, dH/dz + i*Dx)   (spectrum.compute:236)
__device__ __forceinline__ CPair pack_height(float2 H, const KVec& q)
{
  float hx = H.x, hy = H.y;
  float dhdx_x = q.kx * (-hy), dhdx_y = q.kx * hx;
  float dhdz_x = q.kz * (-hy), dhdz_y = q.kz * hx;
  float disX_x = q.dirx * (-hy), disX_y = q.dirx * hx;
  return {f2v{hx - dhdx_y, dhdz_x - disX_y}, f2v{hy + dhdx_x, dhdz_y + disX_x}};
}

// displacementMap texel = (Dz + i*dDx/dx, dDz/dz + i*dDx/dz)   (spectrum.compute:237)
__device__ __forceinline__ CPair pack_displacement(float2 H, const KVec& q)
{
  float hx = H.x, hy = H.y;
  float disZ_x = q.dirz * (-hy), disZ_y = q.dirz * hx;
  float a = -q.kx * q.dirx, b = -q.kz * q.dirz, c = -q.kz * q.dirx;
  float dDXdx_x = a * hx, dDXdx_y = a * hy;
  float dDZdz_x = b * hx, dDZdz_y = b * hy;
  float dDXdz_x = c * hx, dDXdz_y = c * hy;
  return {f2v{disZ_x - dDXdx_y, dDZdz_x - dDXdz_y}, f2v{disZ_y + dDXdx_x, dDZdz_y + dDXdz_x}};
}

// The Nyquist-row term of texel idx = c n + x (k_half_nyquist, ocean_kernels.hip, for its meaning and
// arguments; k_cols_half NYQ runs it in pass 1's least-loaded workgroup instead of a launch of its
// own). Unfused float expressions, so every caller rounds alike whatever it is inlined into (the slab
// paths' kernel and the whole grid's pass 1 must give the same bits).
__device__ __forceinline__ void half_nyquist_texel(const FrameParams& fp, int n, int blk, const float4* __restrict__ h0,
                                                   float4* __restrict__ spec, const float4* __restrict__ h0row,
                                                   int copies, size_t copy_stride,
                                                   const SpectrumConsts* __restrict__ seed,
                                                   const uint64_t* __restrict__ dst, size_t dst_off, int idx)
{
#pragma clang fp contract(off)
  const float dim = (float)n;
  const int c = idx / n, x = idx - c * n;
  float4 s01 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), s23 = s01;
  if (x > 0 && x < n / 2)
  {
    const CascadeFrame f = fp.c[c];
    const int xp = n - x;  // u' = n/2 - x > 0 at column n/2 + u' = n - x; its mirror is x itself
    const float4* hc = h0 + (size_t)c * n * n;
    float4 ap, an;  // row y = 0 (v = -n/2)
    if (seed)
    {
      ap = seed_texel(seed[c], xp, 0, dim);
      an = seed_texel(seed[c], x, 0, dim);
    }
    else
    {
      ap = h0row ? h0row[(size_t)c * n + xp] : hc[(size_t)(xp / blk) * n * blk + (xp % blk)];
      an = h0row ? h0row[(size_t)c * n + x] : hc[(size_t)(x / blk) * n * blk + (x % blk)];
    }
    const KVec qp = make_kvec(xp, 0, dim, f.dk), qn = make_kvec(x, 0, dim, f.dk);
    const float2 hp = evolve(ap, qp.k, f), hn = evolve(an, qn.k, f);
    const float2 dm = make_float2(hn.x - hp.x, hn.y + hp.y);  // Hn - conj(Hp)
    const float2 dq = make_float2(hn.x + hp.x, hn.y - hp.y);  // Hn + conj(Hp)
    const float kz = qn.kz, inv = qn.inv, dirz = qn.dirz, kx = qn.kx;
    const float2 dA = dm;                                              // s = +1
    const float2 dB = make_float2(kz * dq.x, kz * dq.y);               // s = -1
    const float2 dC = make_float2(inv * dm.x, inv * dm.y);             // s = +1
    const float2 dD = make_float2(dirz * dq.x, dirz * dq.y);           // s = -1
    const float2 dE = make_float2(kz * dirz * dm.x, kz * dirz * dm.y); // s = +1
    const float kx2 = kx * kx;
    s01 = make_float4((1.0f - kx) * dA.x, (1.0f - kx) * dA.y, -dB.y - kx * dC.x, dB.x - kx * dC.y);
    s23 = make_float4(-(dD.y - kx2 * dC.y), dD.x - kx2 * dC.x, -dE.x + kx * dD.y, -dE.y - kx * dD.x);
  }
  for (int k = 0; k < copies; k++)
  {
    float4* sp = reinterpret_cast<float4*>(dst ? reinterpret_cast<unsigned char*>(dst[k]) + dst_off
                                               : reinterpret_cast<unsigned char*>(spec) + k * copy_stride);
    sp[((size_t)c * 2 + 0) * n + x] = s01;
    sp[((size_t)c * 2 + 1) * n + x] = s23;
  }
}

}  // namespace oceanfft
