// device/spectrum.h — h0(k) seeding math: Hash, Box-Muller, JONSWAP, Hasselmann / Longuet-Higgins spreading
// (resources/spectrum.compute:29-155), with the settings-only terms evaluated on the host.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ocean_internal.h"

namespace oceanfft
{

// ------------------------------------------------------------------------------------------------
// Constants (resources/spectrum.compute:4, :34-35; resources/fft.compute:14 rounds to the same float)
// ------------------------------------------------------------------------------------------------
#define OCEAN_PI 3.14159265358f
static constexpr float kSigmaSurface = 0.072f;
static constexpr float kRhoWater = 1000.0f;

// ------------------------------------------------------------------------------------------------
// Spectrum math — float32 restatement of resources/spectrum.compute, same operation order.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t hash_raw(uint32_t x, uint32_t y)
{
  // spectrum.compute:109-114
  uint32_t h32 = y + 374761393u + x * 3266489917u;
  h32 = 2246822519u * (h32 ^ (h32 >> 15));
  h32 = 3266489917u * (h32 ^ (h32 >> 13));
  return h32 ^ (h32 >> 16);
}

__device__ __forceinline__ float2 hash_uniform(uint32_t x, uint32_t y)
{
  // spectrum.compute:115-116
  uint32_t n = hash_raw(x, y);
  uint32_t rz1 = n * 48271u;
  return make_float2((float)((n >> 1) & 0x7FFFFFFFu) / (float)0x7FFFFFFF,
                     (float)((rz1 >> 1) & 0x7FFFFFFFu) / (float)0x7FFFFFFF);
}

// Settings-only terms of GetSpectrumAmplitude, evaluated once per launch on the host with the
// oracle's fp32 expressions and glibc powf (bit-identical to the reference restatement) instead of
// once per evaluation on the device.
struct SpectrumConsts
{
  float dk, half_dim, theta_0, g, h;
  float alpha_g2;     // alpha * g * g (spectrum.compute:62, :70)
  float omega_p;      // 22 (g^2 / (U F))^0.333 (spectrum.compute:143)
  float sqrt_h_g;     // sqrt(h / g) (spectrum.compute:74)
  float hassel_hi;    // exponent of the w > w_p branch (spectrum.compute:100)
  float swell2;       // swell * swell
  float spread, spread_2pi;
  float c;            // 0.1 * scale
  float seed_x, seed_y;
  float sigma_rho;    // sigma_surface / rho_water
};

inline SpectrumConsts spectrum_consts(const OceanSettings& s, int n)
{
  SpectrumConsts q;
  q.dk = 2.0f * OCEAN_PI / s.planeSize;
  q.half_dim = (float)n / 2.0f;
  q.theta_0 = s.theta_0;
  q.g = s.g;
  q.h = s.h;
  const float alpha = 0.076f * powf(s.U_10 * s.U_10 / (s.F * s.g), 0.22f);
  q.alpha_g2 = alpha * s.g * s.g;
  q.omega_p = 22.0f * powf(s.g * s.g / (s.U_10 * s.F), 0.333f);
  q.sqrt_h_g = sqrtf(s.h / s.g);
  q.hassel_hi = -2.33f - 1.45f * (s.U_10 * q.omega_p / s.g - 1.17f);
  q.swell2 = s.swell * s.swell;
  q.spread = s.spread;
  q.spread_2pi = s.spread / (2.0f * OCEAN_PI);
  q.c = 0.1f * s.scale;
  q.seed_x = (float)s.seed[0];
  q.seed_y = (float)s.seed[1];
  q.sigma_rho = kSigmaSurface / kRhoWater;
  return q;
}

// Fast transcendentals for the spectrum (tolerance: h0 within 1e-5 of max|h0|, tests/parity.py):
// hardware v_log_f32 / v_exp_f32 (log2 / exp2, ~1 ulp) build pow, exp and log; tanh and sech come
// from one exp each, with an odd series where 1 - 2/(1 + e^2x) would cancel.
__device__ __forceinline__ float log2_hw(float x) { return __builtin_amdgcn_logf(x); }
__device__ __forceinline__ float exp2_hw(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float exp_hw(float x) { return exp2_hw(x * 1.44269504088896341f); }
__device__ __forceinline__ float pow_pos(float x, float y) { return exp2_hw(y * log2_hw(x)); }  // x >= 0, y > 0 or x > 0
__device__ __forceinline__ float rcp_hw(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float tanh_pos(float x)  // x >= 0
{
  if (x < 0.125f)
  {
    const float x2 = x * x;
    return x * fmaf(fmaf(fmaf(-17.0f / 315.0f, x2, 2.0f / 15.0f), x2, -1.0f / 3.0f), x2, 1.0f);
  }
  return 1.0f - 2.0f * rcp_hw(1.0f + exp_hw(2.0f * x));
}

// GetSpectrumAmplitude (spectrum.compute:129-155) at grid index (tx, ty), same formula and order of
// the reference with the settings-only terms hoisted (SpectrumConsts).
__device__ __forceinline__ float2 spectrum_amplitude(const SpectrumConsts& q, float tx, float ty)
{
  // No FMA contraction: the same expression then rounds the same way in every kernel it is inlined
  // into (the pairs kernel, the slab kernel, the fused re-seed column pass), as in the oracle.
#pragma clang fp contract(off)
  const float kx = (tx - q.half_dim) * q.dk;
  const float ky = (ty - q.half_dim) * q.dk;
  const float k2 = kx * kx + ky * ky;
  if (k2 == 0.0f)
    return make_float2(0.0f, 0.0f);
  const float k = __builtin_amdgcn_sqrtf(k2);
  const float theta = atan2f(ky, kx) - q.theta_0;

  // Dispersion (spectrum.compute:38-44)
  const float kh = k * q.h;
  const float tanhKH = kh >= 2.0f * OCEAN_PI ? 1.0f : tanh_pos(kh);
  const float gk_sk3 = q.g * k + q.sigma_rho * k * k * k;
  const float omega = __builtin_amdgcn_sqrtf(gk_sk3 * tanhKH);
  const float rw = rcp_hw(omega);

  // JONSWAP (spectrum.compute:60-78)
  const float w_p = q.omega_p;
  const float sigma = omega > w_p ? 0.09f : 0.07f;
  const float diff = omega - w_p;
  const float r = exp_hw(-diff * diff * rcp_hw(2.0f * sigma * sigma * w_p * w_p));
  const float ratio = w_p * rw, ratio2 = ratio * ratio;
  const float rw2 = rw * rw;
  const float S = q.alpha_g2 * (rw2 * rw2 * rw) * exp_hw(-1.25f * (ratio2 * ratio2)) *
                  exp2_hw(r * 1.72246602447109f);  // 3.3^r, log2(3.3)
  const float w_h = fminf(omega * q.sqrt_h_g, 2.0f);
  float t = fminf(fmaxf(w_h * (1.0f / 2.2f), 0.0f), 1.0f);
  const float Sj = S * (t * t * (3.0f - 2.0f * t));

  // Hasselmann + Longuet-Higgins spreading (spectrum.compute:81-106)
  const float p = omega * rcp_hw(w_p);
  const float sp = omega <= w_p ? 6.97f * pow_pos(p, 4.06f) : 9.77f * pow_pos(p, q.hassel_hi);
  const float sh = sp + 16.0f * tanh_pos(w_p * rw) * q.swell2;
  const float lh = sh < 0.4f ? (0.5f / OCEAN_PI) + sh * (0.220636f + sh * (-0.109f + sh * 0.090f))
                             : 0.56418958354775628f * (0.5f * __builtin_amdgcn_sqrtf(sh) + 0.0625f * __builtin_amdgcn_rsqf(sh));
  // |cos(theta/2)|^(2 sh): near the anti-wind direction cos -> 0 and the power amplifies its relative
  // error, so cos is ocml's accurate cosf (theta/2 is ~10-15 rad with theta_0 = 25, :135), not the
  // hardware v_cos_f32 whose absolute error is a large relative error there.
  const float ct = fabsf(cosf(theta * 0.5f));
  const float d = (1.0f - q.spread) * (lh * pow_pos(ct, 2.0f * sh)) + q.spread_2pi;

  // DispersionDerivative (spectrum.compute:50-57), sech = 2 e^-x / (1 + e^-2x)
  const float em = exp_hw(-q.h * k);
  const float sech = 2.0f * em * rcp_hw(1.0f + em * em);
  const float deriv = (q.h * gk_sk3 * sech * sech + omega * omega) * (0.5f * rw);
  const float chain = deriv * rcp_hw(k) * q.dk * q.dk;

  // Hash + Box-Muller (spectrum.compute:109-127, :153): uvec2(thread + seed)
  const float2 u = hash_uniform((uint32_t)(int64_t)(tx + q.seed_x), (uint32_t)(int64_t)(ty + q.seed_y));
  // accurate logf: for u near 1 the hardware log2's absolute error is a large relative error
  const float rad = __builtin_amdgcn_sqrtf(-2.0f * logf(u.x));
  // sin/cos of the reference's own fp32 argument 2 pi u.y (spectrum.compute:153), accurate (ocml's
  // small-argument path): the hardware v_sin_f32 / v_cos_f32 on u.y in revolutions are as close to
  // the exact values, but their errors are biased, and a bias in every texel's phase adds up over
  // the N^2 texels where the frame sums them in phase (the grid origin, each image row 0 / column 0)
  // while the signal adds up incoherently: 1.3e-4 of the origin's value in a slope channel's spectrum
  // sum at 4096^2, 1.5-1.9e-5 in the frame (tools/parity_probe.py).
  const float th = 2.0f * OCEAN_PI * u.y;
  const float sn = sinf(th), cs = cosf(th);
  const float amp = __builtin_amdgcn_sqrtf(2.0f * Sj * d * chain);
  return make_float2(q.c * (rad * cs) * amp, q.c * (rad * sn) * amp);
}

// One h0 texel evaluated in place: (h0(k), conj(h0(-k))), -k at index N - i
// (spectrum.compute:160-168), with the evaluator and arguments of k_generate_spectrum(_pairs) (ocean_kernels.hip).
__device__ __forceinline__ float4 seed_texel(const SpectrumConsts& q, int x, int y, float dim)
{
  const float2 a = spectrum_amplitude(q, (float)x, (float)y);
  const float2 c = spectrum_amplitude(q, dim - (float)x, dim - (float)y);
  return make_float4(a.x, a.y, c.x, -c.y);
}

}  // namespace oceanfft
