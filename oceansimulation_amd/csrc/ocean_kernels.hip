// ocean_kernels.hip — gfx950 device code for the ocean hot path:
//   h0(k) JONSWAP seeding  ->  h(k,t) evolution fused into the row iFFT  ->  column iFFT + foam.
//
// Reference semantics (paths relative to the reference root):
//   spectrum seeding      resources/spectrum.compute:38-172   (generateSpectrum)
//   evolve + packing      resources/spectrum.compute:183-240  (prepareFFT)
//   2D inverse FFT        resources/fft.compute:21-88 driven by src/FFTCalculator.cpp:73-114
//                         == N^2 * ifft2(ifftshift(X)) per complex lane, no normalisation
//   Jacobian / foam       resources/spectrum.compute:246-259
//
// MI355X design (DESIGN.md has the byte accounting):
//   * 2 HBM passes per frame. Row pass: read h0 (16 B/texel), evolve in registers, 4 complex fields
//     transformed along x, write heightMap + displacementMap rows (32 B). Column pass: read each
//     image's column strips (16 B), transform along y, write back in place (16 B), and for the
//     displacement image write the Jacobian (4 B). 116 B per height-field point.
//   * Each 1D transform is a self-sorting Stockham FFT: one radix-16 butterfly per thread per
//     stage held in VGPRs (16 points x 1-2 complex lanes), LDS only for the exchange between
//     stages (N = 4096 = 16^3 -> 2 exchanges). fftShift is folded into the load index; no
//     bit-reversal pass exists.
//   * Twiddles: exact (host-double-rounded) two-level table in LDS, w = A[e>>LB] * B[e & mask].
//   * Column pass: a strip of C texel columns per workgroup, 4 lanes per row segment (64 B at
//     N = 4096); strips 2m and 2m+1 are given to blocks b and b+8 (same XCD under the observed
//     round-robin placement) so both halves of each 128-B line are consumed from one L2.
//   * Persistent grids sized from occupancy; every loop has a plain item-count exit.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <mutex>
#include <vector>

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

SpectrumConsts spectrum_consts(const OceanSettings& s, int n)
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
  const float ct = fabsf(__builtin_amdgcn_cosf(theta * (0.5f * 0.15915494309189533577f)));  // cos(theta/2)
  const float d = (1.0f - q.spread) * (lh * pow_pos(ct, 2.0f * sh)) + q.spread_2pi;

  // DispersionDerivative (spectrum.compute:50-57), sech = 2 e^-x / (1 + e^-2x)
  const float em = exp_hw(-q.h * k);
  const float sech = 2.0f * em * rcp_hw(1.0f + em * em);
  const float deriv = (q.h * gk_sk3 * sech * sech + omega * omega) * (0.5f * rw);
  const float chain = deriv * rcp_hw(k) * q.dk * q.dk;

  // Hash + Box-Muller (spectrum.compute:109-127, :153): uvec2(thread + seed)
  const float2 u = hash_uniform((uint32_t)(int64_t)(tx + q.seed_x), (uint32_t)(int64_t)(ty + q.seed_y));
  const float rad = __builtin_amdgcn_sqrtf(-2.0f * 0.69314718055994531f * log2_hw(u.x));
  const float sn = __builtin_amdgcn_sinf(u.y), cs = __builtin_amdgcn_cosf(u.y);  // angle 2 pi u.y
  const float amp = __builtin_amdgcn_sqrtf(2.0f * Sj * d * chain);
  return make_float2(q.c * (rad * cs) * amp, q.c * (rad * sn) * amp);
}

// generateSpectrum (spectrum.compute:157-172): texel = (h0(k), conj(h0(-k))), -k taken as N - i.
// Stored strip-blocked, h0[xb][y][blk] (blk texel columns per strip, see ColFirstCfg), so the
// column pass reads each strip as one contiguous run. The reference keeps this image private
// (src/Generator.h:86), so its layout is internal.
__global__ __launch_bounds__(256) void k_generate_spectrum(SpectrumConsts s, int n, int blk, int x0, int width,
                                                          float4* __restrict__ h0)
{
  // columns [x0, x0 + width) of the N x N spectrum (a rank's column slab; width = n for a whole grid)
  const int64_t total = (int64_t)width * n;
  const float dim = (float)n;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x)
  {
    // idx enumerates the blocked layout: b fastest, then y, then xb
    const int b = (int)(idx % blk);
    const int64_t rest = idx / blk;
    const int y = (int)(rest % n), xb = (int)(rest / n);
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
__global__ __launch_bounds__(256) void k_generate_spectrum_pairs(SpectrumConsts s, int n, int blk,
                                                                float4* __restrict__ h0)
{
  const int half = n / 2;
  const int64_t pairs = (int64_t)n * half, total = pairs + n + (half - 1);
  const float dim = (float)n;
  auto at = [&](int x, int y) { return ((int64_t)(x / blk) * n + y) * blk + (x % blk); };
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x)
  {
    int x, y;
    bool mirror;
    if (idx < pairs)  // blocked order over the lower half: b fastest, then y, then xb
    {
      const int b = (int)(idx % blk);
      const int64_t rest = idx / blk;
      y = (int)(rest % half);
      x = (int)(rest / half) * blk + b;
      mirror = x > 0 && y > 0;
    }
    else if (idx < pairs + n)
    {
      x = (int)(idx - pairs);
      y = half;
      mirror = false;
    }
    else
    {
      x = 0;
      y = half + 1 + (int)(idx - pairs - n);
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

// ------------------------------------------------------------------------------------------------
// Buffer (SRD) global access: wave-uniform base in SGPRs + one 32-bit lane offset (T8 in the CDNA
// guide). Keeps the 16 per-thread element addresses out of VGPRs. Offsets stay < 2^31 bytes.
// ------------------------------------------------------------------------------------------------
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t srd(const void* base, int num_bytes)
{
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, num_bytes, 0x00020000);
}

// Raw-buffer range checking: a load at or past num_bytes returns 0 and a store there is dropped,
// which handles ragged row blocks without branches.
constexpr int kAllBytes = 0x7FFFFFFF;

// AUX: cache-policy bits of the buffer instruction (0 = default; 2 = nt, streaming / non-temporal).
template <int AUX = 0>
__device__ __forceinline__ float4 ld4(const void* base, int voff_bytes, int num_bytes = kAllBytes)
{
  f4v r = __builtin_amdgcn_raw_buffer_load_b128(srd(base, num_bytes), voff_bytes, 0, AUX);
  return make_float4(r.x, r.y, r.z, r.w);
}

template <int AUX = 0>
__device__ __forceinline__ void st4(void* base, int voff_bytes, float4 v, int num_bytes = kAllBytes)
{
  f4v r = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(r, srd(base, num_bytes), voff_bytes, 0, AUX);
}

template <int AUX = 0>
__device__ __forceinline__ void st1(void* base, int voff_bytes, float v)
{
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), srd(base, kAllBytes), voff_bytes, 0, AUX);
}

__device__ __forceinline__ int clamp_bytes(int64_t b)
{
  return b > kAllBytes ? kAllBytes : (b < 0 ? 0 : (int)b);
}

// ------------------------------------------------------------------------------------------------
// Complex helpers. V is float2 (one complex lane) or float4 (two lanes: xy, zw), as in the
// reference's packed RGBA32F images (fft.compute:83-84 transforms xy and zw independently).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float2 operator+(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 operator-(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float4 operator+(float4 a, float4 b)
{
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 operator-(float4 a, float4 b)
{
  return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
}
// multiply by +i (inverse-transform sign)
__device__ __forceinline__ float2 mul_i(float2 a) { return make_float2(-a.y, a.x); }
__device__ __forceinline__ float4 mul_i(float4 a) { return make_float4(-a.y, a.x, -a.w, a.z); }
// multiply by -i
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }
__device__ __forceinline__ float4 mul_mi(float4 a) { return make_float4(a.y, -a.x, a.w, -a.z); }
__device__ __forceinline__ float2 cmul(float2 a, float2 w)
{
  return make_float2(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x);
}
__device__ __forceinline__ float4 cmul(float4 a, float2 w)
{
  return make_float4(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x, a.z * w.x - a.w * w.y,
                     a.z * w.y + a.w * w.x);
}

// Two complex lanes in split planes: re = (re0, re1), im = (im0, im1). Every FFT add/sub and
// twiddle multiply is then one v_pk_{add,mul,fma}_f32 over both lanes (the twiddle's parts are
// op_sel splats; multiplying by +-i is operand renaming plus a neg modifier), half the VALU issue
// of the interleaved float4 form. The reference layout (re0, im0, re1, im1) is converted only at
// global loads/stores of caller-visible images; the generator's intermediate stays split.
typedef float f2v __attribute__((ext_vector_type(2)));
struct __attribute__((aligned(16))) CPair
{
  f2v re, im;
};
__device__ __forceinline__ CPair operator+(CPair a, CPair b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ CPair operator-(CPair a, CPair b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ CPair mul_i(CPair a) { return {-a.im, a.re}; }
__device__ __forceinline__ CPair mul_mi(CPair a) { return {a.im, -a.re}; }
__device__ __forceinline__ CPair cmul(CPair a, float2 w)
{
  const f2v wx = {w.x, w.x}, wy = {w.y, w.y};
  return {a.re * wx - a.im * wy, a.re * wy + a.im * wx};
}
// reference texel (re0, im0, re1, im1) <-> split planes
__device__ __forceinline__ CPair to_pair(float4 t) { return {f2v{t.x, t.z}, f2v{t.y, t.w}}; }
__device__ __forceinline__ float4 from_pair(CPair c) { return make_float4(c.re.x, c.im.x, c.re.y, c.im.y); }
// the split texel as raw 16 bytes (re0, re1, im0, im1), for the generator's intermediate
__device__ __forceinline__ CPair raw_pair(float4 t) { return {f2v{t.x, t.y}, f2v{t.z, t.w}}; }
__device__ __forceinline__ float4 pair_raw(CPair c) { return make_float4(c.re.x, c.re.y, c.im.x, c.im.y); }
// the two float2 halves a SPLIT LDS exchange moves one at a time
__device__ __forceinline__ float2 half_of(float4 v, int h) { return h ? make_float2(v.z, v.w) : make_float2(v.x, v.y); }
__device__ __forceinline__ float2 half_of(CPair v, int h) { return h ? make_float2(v.im.x, v.im.y) : make_float2(v.re.x, v.re.y); }
__device__ __forceinline__ void set_half(float4& v, int h, float2 r)
{
  if (h)
    v.z = r.x, v.w = r.y;
  else
    v.x = r.x, v.y = r.y;
}
__device__ __forceinline__ void set_half(CPair& v, int h, float2 r)
{
  if (h)
    v.im = f2v{r.x, r.y};
  else
    v.re = f2v{r.x, r.y};
}

// ------------------------------------------------------------------------------------------------
// Small inverse DFTs (sign +): X[k] = sum_n x[n] exp(+2 pi i n k / r)
// ------------------------------------------------------------------------------------------------
template <typename V>
__device__ __forceinline__ void idft2(V& a0, V& a1)
{
  V t = a0 - a1;
  a0 = a0 + a1;
  a1 = t;
}

template <typename V>
__device__ __forceinline__ void idft4(V& a0, V& a1, V& a2, V& a3)
{
  V s0 = a0 + a2, d0 = a0 - a2, s1 = a1 + a3, d1 = a1 - a3;
  a0 = s0 + s1;
  a2 = s0 - s1;
  a1 = d0 + mul_i(d1);
  a3 = d0 - mul_i(d1);
}

// In: v[n], n = 0..7. Out: v[k] = X[k] (natural order).
template <typename V>
__device__ __forceinline__ void idft8(V* v)
{
  const float R2 = 0.70710678118654752f;
  // n = 2*n1 + n2: DFT4 over n1 for n2 = 0, 1
  idft4(v[0], v[2], v[4], v[6]);
  idft4(v[1], v[3], v[5], v[7]);
  // Y[n2=1][k1] *= W8^k1 (inverse)
  v[3] = cmul(v[3], make_float2(R2, R2));
  v[5] = mul_i(v[5]);
  v[7] = cmul(v[7], make_float2(-R2, R2));
  // DFT2 over n2: X[k1] = Y0[k1] + Y1[k1], X[k1 + 4] = Y0[k1] - Y1[k1]
  V y00 = v[0], y01 = v[2], y02 = v[4], y03 = v[6];
  V y10 = v[1], y11 = v[3], y12 = v[5], y13 = v[7];
  v[0] = y00 + y10;
  v[4] = y00 - y10;
  v[1] = y01 + y11;
  v[5] = y01 - y11;
  v[2] = y02 + y12;
  v[6] = y02 - y12;
  v[3] = y03 + y13;
  v[7] = y03 - y13;
}

// In: v[n], n = 0..15. Out: v[k] = X[k] (natural order). 4 x 4 decomposition.
template <typename V>
__device__ __forceinline__ void idft16(V* v)
{
  const float C1 = 0.92387953251128674f;  // cos(pi/8)
  const float S1 = 0.38268343236508977f;  // sin(pi/8)
  const float R2 = 0.70710678118654752f;
  // n = 4*n1 + n2: DFT4 over n1 for each n2 -> Y[n2][k1] at v[4*k1 + n2]
  idft4(v[0], v[4], v[8], v[12]);
  idft4(v[1], v[5], v[9], v[13]);
  idft4(v[2], v[6], v[10], v[14]);
  idft4(v[3], v[7], v[11], v[15]);
  // twiddle Y[n2][k1] *= W16^(n2*k1), inverse sign
  v[5] = cmul(v[5], make_float2(C1, S1));     // n2=1,k1=1: W^1
  v[9] = cmul(v[9], make_float2(R2, R2));     // n2=1,k1=2: W^2
  v[13] = cmul(v[13], make_float2(S1, C1));   // n2=1,k1=3: W^3
  v[6] = cmul(v[6], make_float2(R2, R2));     // n2=2,k1=1: W^2
  v[10] = mul_i(v[10]);                       // n2=2,k1=2: W^4
  v[14] = cmul(v[14], make_float2(-R2, R2));  // n2=2,k1=3: W^6
  v[7] = cmul(v[7], make_float2(S1, C1));     // n2=3,k1=1: W^3
  v[11] = cmul(v[11], make_float2(-R2, R2));  // n2=3,k1=2: W^6
  v[15] = cmul(v[15], make_float2(-C1, -S1)); // n2=3,k1=3: W^9
  // DFT4 over n2 for each k1: X[k1 + 4*k2]
  idft4(v[0], v[1], v[2], v[3]);
  idft4(v[4], v[5], v[6], v[7]);
  idft4(v[8], v[9], v[10], v[11]);
  idft4(v[12], v[13], v[14], v[15]);
  // now v[4*k1 + k2] = X[k1 + 4*k2]; transpose the 4x4 index to natural order
  V t;
  t = v[1], v[1] = v[4], v[4] = t;
  t = v[2], v[2] = v[8], v[8] = t;
  t = v[3], v[3] = v[12], v[12] = t;
  t = v[6], v[6] = v[9], v[9] = t;
  t = v[7], v[7] = v[13], v[13] = t;
  t = v[11], v[11] = v[14], v[14] = t;
}

// ------------------------------------------------------------------------------------------------
// Stockham radix-16 FFT of length N = 2^LOGN held by T = N/16 cooperating threads.
// Thread i owns v[m] = x[i + m*T]. Stage with radix r and span p (Bainville's formulation):
//   butterfly b, k = b mod p: inputs x[b + t*N/r], twiddle exp(+2 pi i t k / (r p)),
//   outputs y[(b/p)*r*p + k + t*p].
// The first stage uses radix R0 = 2^(LOGN mod 4) (or 16) with p = 1; the rest are radix 16.
// After the last stage (p = T) thread i holds X[i + m*T] directly — no final exchange.
// ------------------------------------------------------------------------------------------------
template <int LOGN>
struct FftShape
{
  static constexpr int N = 1 << LOGN;
  static constexpr int T = N >> 4;
  static constexpr int LOG_R0 = (LOGN & 3) ? (LOGN & 3) : 4;
  static constexpr int R0 = 1 << LOG_R0;
  static constexpr int NSTAGE = 1 + (LOGN - LOG_R0) / 4;
  static constexpr int PADDED = N + N / 16;  // one pad slot per 16: conflict-free Stockham writes
  static constexpr int LB = LOGN / 2;        // two-level twiddle table split
  static constexpr int TB = 1 << LB;
  static constexpr int TA = N >> LB;
  static constexpr int TW_ENTRIES = TA + TB;
};

__device__ __forceinline__ int pad16(int a) { return a + (a >> 4); }

// Hide a loop-invariant value from LICM: without this, hipcc hoists ~100 per-thread LDS/global
// address computations out of the persistent loops and spills them to scratch.
__device__ __forceinline__ int opaque(int v)
{
  asm volatile("" : "+v"(v));
  return v;
}

// w = exp(+2 pi i e / N) from the two-level table (exact host-rounded entries, one cmul).
template <int LOGN>
__device__ __forceinline__ float2 twiddle(int e, const float2* __restrict__ tw)
{
  using S = FftShape<LOGN>;
  float2 lo = tw[e & (S::TB - 1)];
  float2 hi = tw[S::TB + (e >> S::LB)];
  return cmul(lo, hi);
}

// v[t] *= w^t for t = 1..15, w = exp(+2 pi i e1 / N). w and w^4 come from the exact table; the
// other powers are products of at most three table values (error <= ~3 ulp), which keeps only a
// handful of twiddles live instead of 30 hoisted LDS reads.
template <int LOGN, typename V>
__device__ __forceinline__ void apply_stage_twiddles(V* v, int e1, const float2* __restrict__ tw)
{
  constexpr int N = 1 << LOGN;
  const float2 w1 = twiddle<LOGN>(e1, tw);
  const float2 w4 = twiddle<LOGN>((4 * e1) & (N - 1), tw);
  const float2 w2 = cmul(w1, w1);
  const float2 w3 = cmul(w2, w1);
  v[1] = cmul(v[1], w1);
  v[2] = cmul(v[2], w2);
  v[3] = cmul(v[3], w3);
  v[4] = cmul(v[4], w4);
  v[5] = cmul(v[5], cmul(w4, w1));
  v[6] = cmul(v[6], cmul(w4, w2));
  v[7] = cmul(v[7], cmul(w4, w3));
  const float2 w8 = cmul(w4, w4);
  v[8] = cmul(v[8], w8);
  v[9] = cmul(v[9], cmul(w8, w1));
  v[10] = cmul(v[10], cmul(w8, w2));
  v[11] = cmul(v[11], cmul(w8, w3));
  const float2 w12 = cmul(w8, w4);
  v[12] = cmul(v[12], w12);
  v[13] = cmul(v[13], cmul(w12, w1));
  v[14] = cmul(v[14], cmul(w12, w2));
  v[15] = cmul(v[15], cmul(w12, w3));
}

// LDS exchange layout. Element a of the transform lives at padded index pa = a + (a >> 4) (one pad
// slot per 16 elements: conflict-free Stockham writes). Region `reg`:
//   row layout (CI == 0):  slot = reg * RSTRIDE + pa, RSTRIDE = PADDED + 4 (the +4 staggers regions
//                          by 8 banks, so lanes that differ only in reg do not collide)
//   column layout (CI > 0): slot = pa * CI + reg (CI columns interleaved)
// Write/read indices are passed as PADDED indices in closed form (base + t*stride where the
// stride is a multiple of 16 elements), so the per-t offsets fold into ds_* immediates instead
// of occupying 16 address VGPRs.
template <int CI, int PADDED>
__device__ __forceinline__ int lds_slot(int reg, int pa)
{
  if constexpr (CI > 0)
    return pa * CI + reg;
  else
    return reg * (PADDED + 4) + pa;
}

template <int LOGN>
__host__ __device__ constexpr int lds_row_slots(int regions)
{
  return regions * (FftShape<LOGN>::PADDED + 4);
}

// Padded index of x[i + m*T] (the next stage's inputs).
template <int LOGN>
__device__ __forceinline__ int read_pidx(int i, int m)
{
  constexpr int T = FftShape<LOGN>::T;
  if constexpr ((T & 15) == 0)
    return pad16(i) + m * (T + T / 16);
  else
    return pad16(i + m * T);
}

#if defined(OCEAN_ABLATE_EXCHANGE) || defined(OCEAN_ABLATE_BARRIER)
__device__ __forceinline__ void touch(float4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }
__device__ __forceinline__ void touch(CPair& v) { asm volatile("" : "+v"(v.re), "+v"(v.im)); }
#endif
#if defined(OCEAN_ABLATE_BARRIER)  // microbench-only timing ablation (results are wrong)
#define XSYNC() asm volatile("" ::: "memory")
#else
#define XSYNC() __syncthreads()
#endif

// Write the 16 stage outputs (padded indices wp(t), region reg_w), barrier, read back the next
// stage's inputs for the thread's (possibly different) position i_r in region reg_r, barrier.
// SPLIT: float4 data exchanged as two float2 lanes through a float2 buffer (half the LDS).
template <int LOGN, int CI, bool SPLIT, typename V, typename WP>
__device__ __forceinline__ void exchange(V* v, int reg_w, int i_r, int reg_r, void* lds_raw, WP wp)
{
  using S = FftShape<LOGN>;
#if defined(OCEAN_ABLATE_EXCHANGE)  // microbench-only timing ablation (results are wrong)
  for (int t = 0; t < 16; t++)
    touch(v[t]);
  return;
#endif
  if constexpr (!SPLIT)
  {
    V* lds = reinterpret_cast<V*>(lds_raw);
#pragma unroll
    for (int t = 0; t < 16; t++)
      lds[lds_slot<CI, S::PADDED>(reg_w, wp(t))] = v[t];
    XSYNC();
#pragma unroll
    for (int m = 0; m < 16; m++)
      v[m] = lds[lds_slot<CI, S::PADDED>(reg_r, read_pidx<LOGN>(i_r, m))];
    XSYNC();
  }
  else
  {
    static_assert(sizeof(V) == 16, "SPLIT exchange is for two-lane data");
    float2* lds = reinterpret_cast<float2*>(lds_raw);
#pragma unroll
    for (int half = 0; half < 2; half++)
    {
#pragma unroll
      for (int t = 0; t < 16; t++)
        lds[lds_slot<CI, S::PADDED>(reg_w, wp(t))] = half_of(v[t], half);
      XSYNC();
#pragma unroll
      for (int m = 0; m < 16; m++)
        set_half(v[m], half, lds[lds_slot<CI, S::PADDED>(reg_r, read_pidx<LOGN>(i_r, m))]);
      XSYNC();
    }
  }
}

// Full 1D inverse FFT (unnormalised) of the transforms held by the workgroup.
// On entry thread holds v[m] = x[i + m*T] of transform `reg`; the first exchange re-deals the data
// so that from then on (and on exit, v[m] = X[i2 + m*T]) the thread is position i2 of transform
// reg2. Any bijection (i, reg) -> (i2, reg2) over the workgroup is valid: it lets the global loads
// and the global stores use different lane mappings for free. Transforms with a single stage
// (N = 16) have no exchange and require i2 == i, reg2 == reg.
template <int LOGN, int CI, bool SPLIT, typename V>
__device__ __forceinline__ void fft_run(V* v, int i, int reg, int i2, int reg2, void* lds,
                                        const float2* __restrict__ tw)
{
  using S = FftShape<LOGN>;
  constexpr int N = S::N, T = S::T, R0 = S::R0;

  // ---- stage 0: radix R0, p = 1 (no twiddles) ----
  if constexpr (R0 == 16)
  {
    idft16(v);
    if constexpr (S::NSTAGE > 1)
    {
      const int base = 17 * i;  // pad16(16 i + t) = 17 i + t
      exchange<LOGN, CI, SPLIT>(v, reg, i2, reg2, lds, [&](int t) { return base + t; });
    }
  }
  else
  {
    constexpr int U = 16 / R0;  // butterflies per thread; butterfly u uses v[u + t*U]
#pragma unroll
    for (int u = 0; u < U; u++)
    {
      V w[R0];
#pragma unroll
      for (int t = 0; t < R0; t++)
        w[t] = v[u + t * U];
      if constexpr (R0 == 2)
        idft2(w[0], w[1]);
      else if constexpr (R0 == 4)
        idft4(w[0], w[1], w[2], w[3]);
      else
        idft8(w);
#pragma unroll
      for (int t = 0; t < R0; t++)
        v[u + t * U] = w[t];
    }
    // output of butterfly b = i + u*T, element t -> y[b*R0 + t]; v index q = u + t*U
    exchange<LOGN, CI, SPLIT>(v, reg, i2, reg2, lds, [&](int q) {
      int u = q % U, t = q / U;
      return pad16((i + u * T) * R0 + t);
    });
  }

  // ---- radix-16 stages (position i2 of transform reg2) ----
  int p = R0;
#pragma unroll
  for (int s = 1; s < S::NSTAGE; s++)
  {
    const int k = i2 & (p - 1);
    const int stride = N / (16 * p);  // twiddle exponent unit for this stage, in 2 pi / N
    apply_stage_twiddles<LOGN>(v, k * stride, tw);
    idft16(v);
    if (s + 1 < S::NSTAGE)
    {
      const int j = (i2 / p) * 16 * p + k;
      const int pp = p;
      if (pp >= 16)
      {
        const int base = pad16(j), st = pp + pp / 16;
        exchange<LOGN, CI, SPLIT>(v, reg2, i2, reg2, lds, [&](int t) { return base + t * st; });
      }
      else
        exchange<LOGN, CI, SPLIT>(v, reg2, i2, reg2, lds, [&](int t) { return pad16(j + t * pp); });
    }
    p *= 16;
  }
}

template <int LOGN, int CI, bool SPLIT, typename V>
__device__ __forceinline__ void fft_run(V* v, int i, int reg, void* lds, const float2* __restrict__ tw)
{
  fft_run<LOGN, CI, SPLIT>(v, i, reg, i, reg, lds, tw);
}

template <int LOGN>
__device__ __forceinline__ void load_twiddles(float2* tw_lds, const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  for (int e = threadIdx.x; e < S::TW_ENTRIES; e += blockDim.x)
    tw_lds[e] = tw_glob[e];
  __syncthreads();
}

// ------------------------------------------------------------------------------------------------
// Evolution + packing, resources/spectrum.compute:183-240.
// ------------------------------------------------------------------------------------------------
struct KVec
{
  float kx, kz, dirx, dirz, k;
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
  float phase = dispersion_evolve(k, f.g, f.h) * f.time;
  float ws, wc;
  sincos_phase(phase, &ws, &wc);
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

// ------------------------------------------------------------------------------------------------
// FFTCalculator::EncodeIFFT path on caller-owned row-major images: row pass then column pass,
// both in place (no work image).
// ------------------------------------------------------------------------------------------------
template <int LOGN>
struct RowCfg
{
  using S = FftShape<LOGN>;
  static constexpr int RPW = S::T >= 256 ? 1 : 256 / S::T;  // rows per workgroup iteration
  static constexpr int WG = S::T * RPW;
  static constexpr bool SPLIT = (S::N * 16 > 96 * 1024);   // float4 exchange would not fit
  static constexpr int LDS_BYTES = lds_row_slots<LOGN>(RPW) * (SPLIT ? 8 : 16);
  // waves per SIMD the LDS budget admits (>= 1): caps VGPRs so registers never limit residency
  static constexpr int WGS_PER_CU = (150 * 1024) / (LDS_BYTES + 2048) < 1 ? 1 : (150 * 1024) / (LDS_BYTES + 2048);
  static constexpr int MIN_WAVES_RAW = WGS_PER_CU * (WG / 64) / 4;
  static constexpr int MIN_WAVES = MIN_WAVES_RAW < 1 ? 1 : (MIN_WAVES_RAW > 8 ? 8 : MIN_WAVES_RAW);
};

// Row pass of a plain EncodeIFFT on packed images [n_images][N][N] float4, in place.
template <int LOGN>
__global__ __launch_bounds__(RowCfg<LOGN>::WG, RowCfg<LOGN>::MIN_WAVES) void k_rows_ifft(
    int n_images, float4* __restrict__ images, const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  using R = RowCfg<LOGN>;
  constexpr int N = S::N, T = S::T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);

  const int rho0 = threadIdx.x / T, i0 = threadIdx.x % T;
  const int total = n_images * N;
  for (int row0 = blockIdx.x * R::RPW; row0 < total; row0 += gridDim.x * R::RPW)
  {
    const int i = opaque(i0), rho = R::RPW == 1 ? 0 : opaque(rho0);
    // rows row0 .. row0+RPW-1 are contiguous: uniform base, lane offset (rho*N + i)*16; the
    // range limit zeroes/drops rows past the last image (ragged tail for small N)
    float4* lines = images + ((size_t)row0 << LOGN);
    const int lim = clamp_bytes((int64_t)(total - row0) * N * 16);
    const int voff = ((rho << LOGN) + i) * 16;
    CPair v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
      v[m] = to_pair(ld4(lines + ((m + 8) & 15) * T, voff, lim));  // fftShift on x folded into the load
    fft_run<LOGN, 0, R::SPLIT>(v, i, rho, xch, tw);
#pragma unroll
    for (int m = 0; m < 16; m++)
      st4(lines + m * T, voff, from_pair(v[m]), lim);
  }
}

// ------------------------------------------------------------------------------------------------
// Column pass: strips of C texel columns, transformed along y in place. FOAM: images with odd
// index are displacement maps of cascade img/2 and also produce the Jacobian
// (spectrum.compute:246-259) into jac[img/2].
// ------------------------------------------------------------------------------------------------
template <int LOGN>
struct ColCfg
{
  using S = FftShape<LOGN>;
  static constexpr int C = S::T >= 1024 ? 1 : (1024 / S::T > 16 ? 16 : 1024 / S::T);
  static constexpr int WG = S::T * C;
  static constexpr int LDS_BYTES = C * S::PADDED * 8;  // float2 (SPLIT) exchange
  static constexpr int STRIPS = S::N / C;
};

// Block -> work-slot map that gives blocks b and b+8 (same XCD under round-robin placement)
// adjacent strips, so both 64-B halves of a 128-B line meet in one L2. Speed only; any placement
// is correct.
__device__ __forceinline__ int xcd_pair_slot(int b, int G)
{
  if ((G & 15) != 0)
    return b;
  int xcd = b & 7, j = b >> 3;
  int pair = xcd * (G >> 4) + (j >> 1);
  return 2 * pair + (j & 1);
}

template <int LOGN>
__global__ __launch_bounds__(ColCfg<LOGN>::WG) void k_cols(int n_images, float4* __restrict__ images,
                                                           const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  using K = ColCfg<LOGN>;
  constexpr int T = S::T, C = K::C;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);

  const int c0 = threadIdx.x % C, i0 = threadIdx.x / C;
  const int total = n_images * K::STRIPS;
  for (int item = xcd_pair_slot(blockIdx.x, gridDim.x); item < total; item += gridDim.x)
  {
    const int c = opaque(c0), i = opaque(i0);
    const int img = item / K::STRIPS, strip = item - img * K::STRIPS;
    const int x = strip * C + c;
    // image rows i + mm*T: uniform base per mm (SGPR), lane offset (i*N + x)*16 shared by all mm
    float4* ibase = images + ((size_t)img << (2 * LOGN));
    const int voff = ((i << LOGN) + x) * 16;
    CPair v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
    {
      // input q = i + m*T sits in row (q + N/2) mod N = i + ((m + 8) mod 16)*T: fftShift on y
      const int mm = (m + 8) & 15;
      v[m] = to_pair(ld4(ibase + ((size_t)(mm * T) << LOGN), voff));
    }
    fft_run<LOGN, C, true>(v, i, c, xch, tw);
#pragma unroll
    for (int m = 0; m < 16; m++)
      st4(ibase + ((size_t)(m * T) << LOGN), voff, from_pair(v[m]));
  }
}

// ------------------------------------------------------------------------------------------------
// Generator path, column-first (2 HBM passes, every global access a >= 256-byte run per wave):
//   h0      [cascade][xb][y][B]                 strip-blocked (written by k_generate_spectrum)
//   pass 1  k_cols_evolve: per strip of B columns: evolve (spectrum.compute:183-240), iFFT along y
//           of both packed images, write inter[cascade][img][xb][y][B] (contiguous runs)
//   pass 2  k_rows_final: per RPW2 rows of one image: read the blocked intermediate (lanes
//           interleaved so 8 lanes cover one 256-byte run of B texels x RPW2 rows), iFFT along x,
//           write the row-major map (the reference's RGBA32F image) and, for displacement maps,
//           the Jacobian (spectrum.compute:246-259).
// The reference transforms rows first (src/FFTCalculator.cpp:19-20); the 2D iFFT is separable, so
// the order changes only rounding (covered by the parity tolerance).
// ------------------------------------------------------------------------------------------------
template <int LOGN>
struct ColFirstCfg
{
  using S = FftShape<LOGN>;
  static constexpr int N = S::N, T = S::T;
  static constexpr int B = T >= 1024 ? 1 : (T >= 512 ? 2 : (T < 4 ? T : 4));  // texels per block row
  static constexpr int SPW_RAW = 256 / (T * B) < 1 ? 1 : 256 / (T * B);
  static constexpr int SPW = SPW_RAW > N / B ? N / B : SPW_RAW;  // strips per pass-1 item
  static constexpr int C1 = B * SPW;                              // columns per pass-1 item
  static constexpr int WG1 = T * C1;
  static constexpr int LDS1 = C1 * S::PADDED * 8;  // float2 (split-lane) exchange
  static constexpr int RPW2_RAW = 256 / T >= 4 ? 256 / T : (1024 / T < 4 ? 1024 / T : 4);
  static constexpr int RPW2 = RPW2_RAW > N ? N : RPW2_RAW;  // rows per pass-2 item
  static constexpr int WG2 = T * RPW2;
  static constexpr int LDS2 = lds_row_slots<LOGN>(RPW2) * 8;
};

// KEEP: how many of the thread's 16 evolved amplitudes H (2 VGPRs each) stay live from the first
// packed image to the second; the rest are re-read from h0 (bytes this workgroup read ~20 us
// earlier) and evolved again. KEEP = 16 does not fit the 128 VGPRs of a 1024-thread workgroup at
// N = 4096 (spills, which cost HBM traffic); KEEP = 4 does (default_keep).
// Cache policy: data touched once per frame (the KEEP once-read h0 texels, every store) is
// streamed non-temporally (LA, SA = kStream: 3-5 % faster per pass than the default policy); the
// twice-read h0 texels use the default policy (LR = 0) so the second read hits the cache
// hierarchy instead of HBM (6 % faster pass 1 than streaming them; tools/microbench/genbench).
constexpr int kStream = 2;

template <int LOGN, int KEEP, int LA = kStream, int SA = kStream, bool NOMEM = false, int LR = 0, bool NOCOMP = false>
__global__ __launch_bounds__(ColFirstCfg<LOGN>::WG1) void k_cols_evolve(
    FrameParams fp, SlabGeom g, const float4* __restrict__ h0, float4* __restrict__ inter,
    const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  using K = ColFirstCfg<LOGN>;
  constexpr int N = S::N, T = S::T, B = K::B, SPW = K::SPW;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);

  const int w = g.w, wb = g.w / B;  // slab columns (= rows per destination block), strips in slab
  const int groups = wb / SPW;      // pass-1 items per cascade
  const int total = fp.cascades * groups;
  const float dim = (float)N;
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    // thread coordinates re-derived from one opaque copy of threadIdx.x (fewer live VGPRs)
    const int tid = opaque((int)threadIdx.x);
    const int b = tid % B, sl = SPW == 1 ? 0 : tid / (B * T);
    const int c = item / groups, xb0 = (item - c * groups) * SPW;
    const CascadeFrame f = fp.c[c];
    // this item's SPW strips of the slab's h0 are one contiguous run of SPW*N*B texels
    const float4* src = h0 + ((size_t)c * wb + xb0) * N * B;
    const int x = g.x0 + (xb0 + sl) * B + b;  // global column (k index)
    float2 H[KEEP > 0 ? KEEP : 1];
#pragma unroll 1
    for (int img = 0; img < 2; img++)
    {
      // keep the k-vector math inside this iteration (see opaque())
      const int i = (opaque((int)threadIdx.x) / B) % T;
      const int voff = ((sl * N + i) * B + b) * 16;
      float4 a[16];
#pragma unroll
      for (int m = 0; m < 16; m++)
        if (img == 0 || m >= KEEP)
        {
          if constexpr (NOMEM)  // compute-only timing variant (microbench): no HBM reads
            a[m] = make_float4(1e-3f * m, 2e-3f * (float)i, 1e-3f * (float)b, 1e-4f * (float)item);
          else if (m < KEEP)  // read once per frame
            a[m] = ld4<LA>(src + ((m + 8) & 15) * T * B, voff);  // fftShift on y folded into the load
          else  // read twice (re-evolved for the second image): policy LR
            a[m] = ld4<LR>(src + ((m + 8) & 15) * T * B, voff);
        }
      CPair v[16];
#pragma unroll
      for (int m = 0; m < 16; m++)
      {
        const int y = i + ((m + 8) & 15) * T;
        KVec q = make_kvec(x, y, dim, f.dk);
        float2 Hm;
        if constexpr (NOCOMP)  // memory-only timing ablation (microbench): no evolution, no FFT
        {
          v[m] = CPair{f2v{a[m].x, a[m].y}, f2v{a[m].z, a[m].w}};
          continue;
        }
        if (img == 1 && m < KEEP)
          Hm = H[m];
        else
          Hm = evolve(a[m], q.k, f);
        if (img == 0 && m < KEEP)
          H[m] = Hm;
        v[m] = img == 0 ? pack_height(Hm, q) : pack_displacement(Hm, q);
      }
      if constexpr (!NOCOMP)
        fft_run<LOGN, K::C1, true>(v, i, sl * B + b, xch, tw);
      // Output rows y = i + m*T go to destination block q = y / w (uniform per m since T | w),
      // laid out inter[c][q][img][xb_local][y - q*w][B]: each destination's block is one
      // contiguous range (what the all-to-all sends; for ranks == 1 it is [c][img][xb][y][B]).
      float4* dst = inter + (size_t)c * 2 * N * w;
      const int soff = ((sl * w + i) * B + b) * 16;
#pragma unroll
      for (int m = 0; m < 16; m++)
      {
        const int q = (m * T) / w, yl = (m * T) % w;
        if constexpr (NOMEM)
          asm volatile("" ::"v"(v[m].re), "v"(v[m].im));
        else  // intermediate texels stay in split form (pair_raw): pass 2 reads them as such
          st4<SA>(dst + (((size_t)(q * 2 + img) * wb + xb0) * w + yl) * B, soff, pair_raw(v[m]));
      }
    }
  }
}

// Standalone EncodeIFFT, column-first with a work image (src/FFTCalculator.cpp keeps a workImage
// too): pass A reads the caller's row-major image in strips of B columns (64-B pieces per row,
// the only strided access), iFFTs along y with the fftShift folded into the row index, and writes
// the blocked split-plane work image work[img][x/B][y][B] contiguously; pass B is k_rows_final on
// it (256-B runs in, row-major rows out, no Jacobian). Measured patterns (profiles/
// r01_colbench_patterns.log): strided read + contiguous write 3.4 TB/s, against 2.1-2.4 TB/s for
// the in-place column pass that reads and writes 64-B pieces.
template <int LOGN>
__global__ __launch_bounds__(ColFirstCfg<LOGN>::WG1) void k_cols_to_blocks(int images, const float4* __restrict__ src_images,
                                                                          float4* __restrict__ work,
                                                                          const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  using K = ColFirstCfg<LOGN>;
  constexpr int N = S::N, T = S::T, B = K::B, SPW = K::SPW;
  static_assert(SPW == 1, "one strip per item");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);
  const int strips = N / B;
  const int total = images * strips;
  // adjacent strips (the two 64-B halves of each 128-B line) on blocks b, b+8: one XCD, one L2
  for (int item = xcd_pair_slot(blockIdx.x, gridDim.x); item < total; item += gridDim.x)
  {
    const int tid = opaque((int)threadIdx.x);
    const int b = tid % B, i = (tid / B) % T;
    const int img = item / strips, xb = item - img * strips;
    // row y = i + mm*T of the input, column xb*B + b: uniform base per m, lane offset (i*N + b)*16
    const float4* src = src_images + ((size_t)img << (2 * LOGN)) + (size_t)xb * B;
    const int voff = ((i << LOGN) + b) * 16;
    CPair v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
      v[m] = to_pair(ld4<kStream>(src + ((size_t)(((m + 8) & 15) * T) << LOGN), voff));  // fftShift on y
    fft_run<LOGN, K::C1, true>(v, i, b, xch, tw);
    float4* dst = work + ((size_t)img << (2 * LOGN)) + (size_t)xb * N * B;
    const int soff = (i * B + b) * 16;
#pragma unroll
    for (int m = 0; m < 16; m++)
      st4<kStream>(dst + m * T * B, soff, pair_raw(v[m]));
  }
}

// BLOCKED: input is pass 1's output after the exchange, inter[c][src][img][xb_local][y][B] for this
// rank's w rows (xb = src * (w/B) + xb_local); otherwise row-major [c][img][y][x] (after
// k_blocks_to_rows, used when B == 1).
// ABL: timing ablations for tools/microbench (results wrong by construction): 1 = no HBM traffic,
// 2 = no FFT (memory traffic and stores only).
template <int LOGN, bool BLOCKED, int LA = kStream, int SA = kStream, int RPW_ = ColFirstCfg<LOGN>::RPW2, int ABL = 0>
__global__ __launch_bounds__(FftShape<LOGN>::T * RPW_) void k_rows_final(
    int images, SlabGeom g, const float4* __restrict__ inter, float4* __restrict__ maps, float* __restrict__ jac,
    FoamParams foam, const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  using K = ColFirstCfg<LOGN>;
  constexpr int N = S::N, T = S::T, B = BLOCKED ? K::B : 1, RPW = RPW_;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);

  const int w = g.w, wb = g.w / B;
  const int blocks = w / RPW;  // pass-2 items per image
  // Loads (blocked input): lanes b fastest, then row r, then ihi, so 16 consecutive lanes read one
  // B*RPW*16-byte run [xb][y0..y0+RPW-1][0..B-1]. After the first exchange the thread becomes
  // position i2 of row r2 with i2 fastest, so each wave stores 64 consecutive texels of one row.
  // Row-major input: i fastest for both.
  const int b0 = threadIdx.x % B, r0 = (threadIdx.x / B) % RPW, ihi0 = threadIdx.x / (B * RPW);
  const int i20 = threadIdx.x % T, r20 = threadIdx.x / T;
  constexpr bool REMAP = BLOCKED && S::NSTAGE > 1;
  const int total = images * blocks;  // images = 2 per cascade (height, displacement)
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    int i, r;
    if constexpr (BLOCKED)
    {
      const int b = opaque(b0), ihi = opaque(ihi0);
      r = RPW == 1 ? 0 : opaque(r0);
      i = ihi * B + b;
    }
    else
    {
      i = opaque(i20);
      r = RPW == 1 ? 0 : opaque(r20);
    }
    const int i2 = REMAP ? opaque(i20) : i, r2 = REMAP ? (RPW == 1 ? 0 : opaque(r20)) : r;
    const int cimg = item / blocks, y0 = (item - cimg * blocks) * RPW;
    const int c = cimg >> 1, img = cimg & 1;
    CPair v[16];
    if constexpr (BLOCKED)
    {
      const float4* src = inter + (size_t)c * 2 * N * w + (size_t)y0 * B;
      const int ihi = i / B, b = i % B;
      const int voff = ((ihi * w + r) * B + b) * 16;
#pragma unroll
      for (int m = 0; m < 16; m++)
      {
        // column block xb = ihi + mm*T/B: source rank and local block are uniform per m
        const int xbm = ((m + 8) & 15) * (T / B);  // fftShift on x
        const int srcr = xbm / wb, xbl = xbm % wb;
        if constexpr (ABL == 1)
          v[m] = CPair{f2v{1e-3f * m, (float)i}, f2v{(float)r, 1e-4f * (float)item}};
        else
          v[m] = raw_pair(ld4<LA>(src + ((size_t)(srcr * 2 + img) * wb + xbl) * w * B, voff));
      }
    }
    else
    {
      const float4* src = inter + ((size_t)cimg * w + y0) * N;
      const int voff = ((r << LOGN) + i) * 16;
#pragma unroll
      for (int m = 0; m < 16; m++)
        v[m] = raw_pair(ld4<LA>(src + ((m + 8) & 15) * T, voff));  // fftShift on x
    }
    if constexpr (ABL != 2)
      fft_run<LOGN, 0, true>(v, i, r, i2, r2, xch, tw);
    float4* dst = maps + ((size_t)cimg * w + y0) * N;
    const int woff = ((r2 << LOGN) + i2) * 16;
#pragma unroll
    for (int m = 0; m < 16; m++)
      if constexpr (ABL == 1)
        asm volatile("" ::"v"(v[m].re), "v"(v[m].im));
      else
        st4<SA>(dst + m * T, woff, from_pair(v[m]));
    if (jac != nullptr && (img & 1))  // jac == nullptr: plain EncodeIFFT (launch_ifft_colfirst)
    {
      // displacementMap (Dz, dDx/dx, dDz/dz, dDx/dz) = (re0, im0, re1, im1): Jacobian,
      // spectrum.compute:246-259
      const float lam = foam.displacement[c];
      float* jb = jac + ((size_t)c * w + y0) * N;
      const int joff = ((r2 << LOGN) + i2) * 4;
#pragma unroll
      for (int m = 0; m < 16; m++)
      {
        const float jv = (1.0f + lam * v[m].im.x) * (1.0f + lam * v[m].re.y) - lam * lam * v[m].im.y * v[m].im.y;
        if constexpr (ABL == 1)
          asm volatile("" ::"v"(jv));
        else
          st1<SA>(jb + m * T, joff, jv);
      }
    }
  }
}

// B == 1 (N = 16384: one 256-KiB column per CU) makes the blocked layout column-major, whose rows
// the row pass could only read 16 bytes at a time. This tiled transpose (64 x 64 texels through
// LDS, 1-KiB runs on both sides) turns inter[c][src][img][x_local][y] into row-major
// out[c][img][y][x] for the rank's w rows.
__global__ __launch_bounds__(256) void k_blocks_to_rows(int cascades, int n, int w, const float4* __restrict__ in,
                                                        float4* __restrict__ out)
{
  __shared__ float4 tile[64][65];
  const int tiles_x = n / 64, tiles_y = w / 64;
  const int total = cascades * 2 * tiles_x * tiles_y;
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    const int cimg = item / (tiles_x * tiles_y), t = item % (tiles_x * tiles_y);
    const int c = cimg >> 1, img = cimg & 1;
    const int tx = t % tiles_x, ty = t / tiles_x;
    // read: 64 columns x 64 rows; column x is contiguous in y
    for (int k = 0; k < 16; k++)
    {
      const int L = k * 256 + threadIdx.x, col = L >> 6, row = L & 63;
      const int x = tx * 64 + col, srcr = x / w, xl = x % w;
      tile[col][row] = in[(size_t)c * 2 * n * w + ((size_t)(srcr * 2 + img) * w + xl) * w + ty * 64 + row];
    }
    __syncthreads();
    for (int k = 0; k < 16; k++)
    {
      const int L = k * 256 + threadIdx.x, row = L >> 6, col = L & 63;
      out[((size_t)cimg * w + ty * 64 + row) * n + tx * 64 + col] = tile[col][row];
    }
    __syncthreads();
  }
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
template <int CH>
__device__ __forceinline__ void sample_linear_repeat(const float* __restrict__ tex, int n, float u, float v, float* out)
{
#pragma clang fp contract(off)
  const float s = u * (float)n - 0.5f, t = v * (float)n - 0.5f;
  const float fs = floorf(s), ft = floorf(t);
  const float a = s - fs, b = t - ft;
  const int m = n - 1;  // n is a power of two: & m is the repeat wrap, also for negative indices
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
    for (int c = 0; c < p.count; c++)
    {
      float d1[4], d2[4];
      const float u = px / p.c[c].plane, v = pz / p.c[c].plane;
      sample_linear_repeat<4>(reinterpret_cast<const float*>(p.c[c].height), p.n, u, v, d1);
      sample_linear_repeat<4>(reinterpret_cast<const float*>(p.c[c].disp), p.n, u, v, d2);
      px += p.c[c].scale * d1[3];
      py += d1[0];
      pz += p.c[c].scale * d2[0];
    }
    float d[4] = {0.0f, 0.0f, 0.0f, 0.0f}, jac = 0.0f;
    for (int c = 0; c < p.count; c++)
    {
      float d1[4], d2[4], j;
      const float u = px / p.c[c].plane, v = pz / p.c[c].plane;
      sample_linear_repeat<4>(reinterpret_cast<const float*>(p.c[c].height), p.n, u, v, d1);
      sample_linear_repeat<4>(reinterpret_cast<const float*>(p.c[c].disp), p.n, u, v, d2);
      sample_linear_repeat<1>(p.c[c].jac, p.n, u, v, &j);
      jac += j / (float)p.count;
      const float f = p.c[c].scale;
      d[0] += d1[1];
      d[1] += d2[1] * f;
      d[2] += d1[2];
      d[3] += d2[2] * f;
    }
    const float sx = d[0] / (1.0f + d[1]), sz = d[2] / (1.0f + d[3]);
    const float nx = -sx, ny = 1.0f, nz = -sz;
    const float len = sqrtf(nx * nx + ny * ny + nz * nz);
    out[2 * idx] = make_float4(px, py, pz, jac);
    out[2 * idx + 1] = make_float4(nx / len, ny / len, nz / len, 0.0f);
  }
}

// ------------------------------------------------------------------------------------------------
// Host-side launchers (dispatch on log2 N).
// ------------------------------------------------------------------------------------------------
template <int LOGN>
static int lds_bytes_rows()
{
  using S = FftShape<LOGN>;
  return ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + RowCfg<LOGN>::LDS_BYTES;
}
template <int LOGN>
static int lds_bytes_cols()
{
  using S = FftShape<LOGN>;
  return ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + ColCfg<LOGN>::LDS_BYTES;
}

template <typename F>
static hipError_t with_logn(int logn, F&& f)
{
  switch (logn)
  {
  case 4: return f(std::integral_constant<int, 4>{});
  case 5: return f(std::integral_constant<int, 5>{});
  case 6: return f(std::integral_constant<int, 6>{});
  case 7: return f(std::integral_constant<int, 7>{});
  case 8: return f(std::integral_constant<int, 8>{});
  case 9: return f(std::integral_constant<int, 9>{});
  case 10: return f(std::integral_constant<int, 10>{});
  case 11: return f(std::integral_constant<int, 11>{});
  case 12: return f(std::integral_constant<int, 12>{});
  case 13: return f(std::integral_constant<int, 13>{});
  case 14: return f(std::integral_constant<int, 14>{});
  default: return hipErrorInvalidValue;
  }
}

// Persistent grid: resident blocks per CU x CUs, capped by the work item count. The occupancy
// query and the dynamic-LDS attribute are set once per kernel instantiation (host API calls cost
// microseconds; a frame is two launches).
struct LaunchCacheEntry
{
  const void* kernel;
  int lds;
  int per_cu;
};

template <typename K>
static int persistent_grid(K kernel, int wg, int lds, int items, int cus)
{
  static std::mutex mu;
  static std::vector<LaunchCacheEntry> cache;
  int per_cu = -1;
  {
    std::lock_guard<std::mutex> lock(mu);
    for (const auto& e : cache)
      if (e.kernel == (const void*)kernel && e.lds == lds)
        per_cu = e.per_cu;
    if (per_cu < 0)
    {
      per_cu = 0;
      (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, wg, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
      cache.push_back({(const void*)kernel, lds, per_cu});
    }
  }
  long g = (long)per_cu * cus;
  if (g > items)
    g = items;
  return g < 1 ? 1 : (int)g;
}

int spectrum_block(int logn)
{
  int t = 1 << (logn - 4);
  return t >= 1024 ? 1 : (t >= 512 ? 2 : (t < 4 ? t : 4));
}

hipError_t launch_generate_spectrum(const OceanSettings& s, int n, float4* h0, hipStream_t stream, int cus, int x0,
                                    int width)
{
  int logn = 0;
  while ((1 << logn) < n)
    logn++;
  if (width <= 0)
    width = n;
  const bool whole = x0 == 0 && width == n;  // a slab's partner columns belong to other ranks
  long total = whole ? (long)n * (n / 2) + n + n / 2 - 1 : (long)n * width;
  long blocks = (total + 255) / 256;
  long cap = (long)cus * 16;
  if (blocks > cap)
    blocks = cap;
  if (whole)
    hipLaunchKernelGGL(k_generate_spectrum_pairs, dim3((unsigned)blocks), dim3(256), 0, stream,
                       spectrum_consts(s, n), n, spectrum_block(logn), h0);
  else
    hipLaunchKernelGGL(k_generate_spectrum, dim3((unsigned)blocks), dim3(256), 0, stream, spectrum_consts(s, n), n,
                       spectrum_block(logn), x0, width, h0);
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
  hipLaunchKernelGGL(k_surface, dim3((unsigned)blocks), dim3(256), 0, stream, p, plane, xz, count, out);
  return hipGetLastError();
}

hipError_t launch_hash(const uint32_t* xy, int count, uint32_t* raw, float2* uv, hipStream_t stream)
{
  hipLaunchKernelGGL(k_hash, dim3((count + 255) / 256), dim3(256), 0, stream, xy, count, raw, uv);
  return hipGetLastError();
}

hipError_t launch_cols_evolve(int logn, const FrameParams& fp, const SlabGeom& g, const float4* h0, float4* inter,
                              const float2* tw, hipStream_t stream, int cus, int keep)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    using K = ColFirstCfg<LOGN>;
    using S = FftShape<LOGN>;
    auto kern = keep >= 16 ? k_cols_evolve<LOGN, 16>
                           : (keep >= 8 ? k_cols_evolve<LOGN, 8> : (keep >= 4 ? k_cols_evolve<LOGN, 4> : k_cols_evolve<LOGN, 0>));
    const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + K::LDS1;
    const int items = fp.cascades * ((g.w / K::B) / K::SPW);
    const int grid = persistent_grid(kern, K::WG1, lds, items, cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG1), lds, stream, fp, g, h0, inter, tw);
    return hipGetLastError();
  });
}

bool ifft_colfirst_supported(int logn) { return logn == 12; }

hipError_t launch_ifft_colfirst(int logn, int n_images, float4* images, float4* work, const float2* tw,
                                hipStream_t stream, int cus)
{
  if (!ifft_colfirst_supported(logn))
    return hipErrorInvalidValue;
  constexpr int LOGN = 12;
  using K = ColFirstCfg<LOGN>;
  using S = FftShape<LOGN>;
  const int tw_bytes = ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  {
    auto kern = k_cols_to_blocks<LOGN>;
    const int lds = tw_bytes + K::LDS1;
    const int grid = persistent_grid(kern, K::WG1, lds, n_images * (S::N / K::B), cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG1), lds, stream, n_images, images, work, tw);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
      return e;
  }
  auto kern = k_rows_final<LOGN, true>;
  const int lds = tw_bytes + K::LDS2;
  const SlabGeom g{0, S::N};
  const int grid = persistent_grid(kern, K::WG2, lds, n_images * (S::N / K::RPW2), cus);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG2), lds, stream, n_images, g, work, images, (float*)nullptr,
                     FoamParams{}, tw);
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

hipError_t launch_rows_final(int logn, int cascades, const SlabGeom& g, const float4* inter, float4* scratch,
                             float4* maps, float* jac, const FoamParams& foam, const float2* tw, hipStream_t stream,
                             int cus)
{
  const bool transpose = rows_need_transpose(logn) && scratch != nullptr;
  if (transpose)
  {
    const int n = 1 << logn;
    const int items = cascades * 2 * (n / 64) * (g.w / 64);
    const int grid = persistent_grid(k_blocks_to_rows, 256, 0, items, cus);
    hipLaunchKernelGGL(k_blocks_to_rows, dim3(grid), dim3(256), 0, stream, cascades, n, g.w, inter, scratch);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
      return e;
  }
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    using K = ColFirstCfg<LOGN>;
    using S = FftShape<LOGN>;
    const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + K::LDS2;
    const int items = cascades * 2 * (g.w / K::RPW2);
    if (transpose)
    {
      auto kern = k_rows_final<LOGN, false>;
      const int grid = persistent_grid(kern, K::WG2, lds, items, cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG2), lds, stream, 2 * cascades, g, scratch, maps, jac, foam, tw);
    }
    else
    {
      auto kern = k_rows_final<LOGN, true>;
      const int grid = persistent_grid(kern, K::WG2, lds, items, cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG2), lds, stream, 2 * cascades, g, inter, maps, jac, foam, tw);
    }
    return hipGetLastError();
  });
}

hipError_t launch_rows_ifft(int logn, int n_images, float4* images, const float2* tw, hipStream_t stream, int cus)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    using R = RowCfg<LOGN>;
    auto kern = k_rows_ifft<LOGN>;
    int lds = lds_bytes_rows<LOGN>();
    int items = ((n_images << LOGN) + R::RPW - 1) / R::RPW;
    int grid = persistent_grid(kern, R::WG, lds, items, cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(R::WG), lds, stream, n_images, images, tw);
    return hipGetLastError();
  });
}

hipError_t launch_cols(int logn, int n_images, float4* images, const float2* tw, hipStream_t stream, int cus)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    using K = ColCfg<LOGN>;
    int lds = lds_bytes_cols<LOGN>();
    int items = n_images * K::STRIPS;
    auto kern = k_cols<LOGN>;
    int grid = persistent_grid(kern, K::WG, lds, items, cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG), lds, stream, n_images, images, tw);
    return hipGetLastError();
  });
}

// A/B hook for tools/microbench/genbench at N = 4096. Pass 1: variant 0/1 = KEEP 0/4 with default
// policy on the twice-read h0, 2 = KEEP 4 all loads default, 3 = KEEP 4 compute only (no HBM). Pass 2: cache policy 0 default, 1 nt stores, 2 nt loads + stores.
hipError_t launch_policy_variant(int pass, int policy, const FrameParams& fp, const SlabGeom& g, const float4* in,
                                 float4* out, float* jac, const FoamParams& foam, const float2* tw, hipStream_t stream,
                                 int cus)
{
  constexpr int LOGN = 12;
  using K = ColFirstCfg<LOGN>;
  using S = FftShape<LOGN>;
  if (pass == 1)
  {
    auto kern = policy == 0 ? k_cols_evolve<LOGN, 0, kStream, kStream, false, 0>
                            : (policy == 1 ? k_cols_evolve<LOGN, 4, kStream, kStream, false, 0>
                                           : (policy == 2 ? k_cols_evolve<LOGN, 4, 0, kStream, false, 0>
                                                          : (policy == 3 ? k_cols_evolve<LOGN, 4, kStream, kStream, true>
                                                                         : k_cols_evolve<LOGN, 4, kStream, kStream, false, 0, true>)));
    const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + K::LDS1;
    const int items = fp.cascades * ((g.w / K::B) / K::SPW);
    const int grid = persistent_grid(kern, K::WG1, lds, items, cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG1), lds, stream, fp, g, in, out, tw);
  }
  else
  {
    // policy 3: 2 rows per workgroup (512 threads, half the LDS: two workgroups per CU);
    // 4 / 5: ablations compute only / memory only
    const int rpw = policy == 3 ? 2 : K::RPW2;
    auto kern = policy == 0 ? k_rows_final<LOGN, true, 0, 0>
                : policy == 1 ? k_rows_final<LOGN, true, 0, 2>
                : policy == 2 ? k_rows_final<LOGN, true, 2, 2>
                : policy == 3 ? k_rows_final<LOGN, true, 2, 2, 2>
                : policy == 4 ? k_rows_final<LOGN, true, 2, 2, K::RPW2, 1>
                              : k_rows_final<LOGN, true, 2, 2, K::RPW2, 2>;
    const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + lds_row_slots<LOGN>(rpw) * 8;
    const int items = fp.cascades * 2 * (g.w / rpw);
    const int grid = persistent_grid(kern, S::T * rpw, lds, items, cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(S::T * rpw), lds, stream, 2 * fp.cascades, g, in, out, jac, foam, tw);
  }
  return hipGetLastError();
}

int twiddle_entries(int logn)
{
  int lb = logn / 2;
  return (1 << lb) + (1 << (logn - lb));
}

}  // namespace oceanfft
