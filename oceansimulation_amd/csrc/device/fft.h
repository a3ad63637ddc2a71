// device/fft.h — the in-register Stockham radix-16 inverse FFT: split-plane packed complex arithmetic,
// small inverse DFTs, twiddles, LDS exchanges (resources/fft.compute:21-88 semantics).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device/memory.h"

namespace oceanfft
{

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

// Exchange ordering. Workgroup transforms: a barrier. WAVE (the transform lives in one wavefront and
// its LDS region is the wave's own): the LDS executes one wave's ds_* instructions in issue order, so
// only the compiler has to keep the writes before the reads (and the reads before the next writes).
template <bool WAVE>
__device__ __forceinline__ void xsync()
{
  if constexpr (WAVE)
  {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  else
    XSYNC();
}

// Write the 16 stage outputs (padded indices wp(t), region reg_w), barrier, read back the next
// stage's inputs for the thread's (possibly different) position i_r in region reg_r, barrier.
// SPLIT: float4 data exchanged as two float2 lanes through a float2 buffer (half the LDS).
// QUARTER (CPair only): the four floats re.x, re.y, im.x, im.y one at a time through a float buffer
// (a quarter of the LDS, twice the split exchange's barriers), so a 1024-thread column workgroup
// leaves room in the LDS for the H it keeps across its field rounds (k_cols_half QX).
template <int LOGN, int CI, bool SPLIT, bool WAVE = false, bool QUARTER = false, typename V, typename WP>
__device__ __forceinline__ void exchange(V* v, int reg_w, int i_r, int reg_r, void* lds_raw, WP wp)
{
  using S = FftShape<LOGN>;
#if defined(OCEAN_ABLATE_EXCHANGE)  // microbench-only timing ablation (results are wrong)
  for (int t = 0; t < 16; t++)
    touch(v[t]);
  return;
#endif
  if constexpr (QUARTER)
  {
    static_assert(sizeof(V) == 16 && SPLIT, "QUARTER exchange is for CPair data");
    float* lds = reinterpret_cast<float*>(lds_raw);
    auto get = [](const CPair& c, int q) { return q == 0 ? c.re.x : q == 1 ? c.re.y : q == 2 ? c.im.x : c.im.y; };
    auto put = [](CPair& c, int q, float x) {
      if (q == 0)
        c.re.x = x;
      else if (q == 1)
        c.re.y = x;
      else if (q == 2)
        c.im.x = x;
      else
        c.im.y = x;
    };
#pragma unroll
    for (int q = 0; q < 4; q++)
    {
#pragma unroll
      for (int t = 0; t < 16; t++)
        lds[lds_slot<CI, S::PADDED>(reg_w, wp(t))] = get(v[t], q);
      xsync<WAVE>();
#pragma unroll
      for (int m = 0; m < 16; m++)
        put(v[m], q, lds[lds_slot<CI, S::PADDED>(reg_r, read_pidx<LOGN>(i_r, m))]);
      xsync<WAVE>();
    }
  }
  else if constexpr (!SPLIT)
  {
    V* lds = reinterpret_cast<V*>(lds_raw);
#pragma unroll
    for (int t = 0; t < 16; t++)
      lds[lds_slot<CI, S::PADDED>(reg_w, wp(t))] = v[t];
    xsync<WAVE>();
#pragma unroll
    for (int m = 0; m < 16; m++)
      v[m] = lds[lds_slot<CI, S::PADDED>(reg_r, read_pidx<LOGN>(i_r, m))];
    xsync<WAVE>();
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
      xsync<WAVE>();
#pragma unroll
      for (int m = 0; m < 16; m++)
        set_half(v[m], half, lds[lds_slot<CI, S::PADDED>(reg_r, read_pidx<LOGN>(i_r, m))]);
      xsync<WAVE>();
    }
  }
}

// Full 1D inverse FFT (unnormalised) of the transforms held by the workgroup.
// On entry thread holds v[m] = x[i + m*T] of transform `reg`; the first exchange re-deals the data
// so that from then on (and on exit, v[m] = X[i2 + m*T]) the thread is position i2 of transform
// reg2. Any bijection (i, reg) -> (i2, reg2) over the workgroup is valid: it lets the global loads
// and the global stores use different lane mappings for free. Transforms with a single stage
// (N = 16) have no exchange and require i2 == i, reg2 == reg.
template <int LOGN, int CI, bool SPLIT, bool WAVE = false, bool QUARTER = false, typename V>
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
      exchange<LOGN, CI, SPLIT, WAVE, QUARTER>(v, reg, i2, reg2, lds, [&](int t) { return base + t; });
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
    exchange<LOGN, CI, SPLIT, WAVE, QUARTER>(v, reg, i2, reg2, lds, [&](int q) {
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
        exchange<LOGN, CI, SPLIT, WAVE, QUARTER>(v, reg2, i2, reg2, lds, [&](int t) { return base + t * st; });
      }
      else
        exchange<LOGN, CI, SPLIT, WAVE, QUARTER>(v, reg2, i2, reg2, lds, [&](int t) { return pad16(j + t * pp); });
    }
    p *= 16;
  }
}

template <int LOGN, int CI, bool SPLIT, typename V>
__device__ __forceinline__ void fft_run(V* v, int i, int reg, void* lds, const float2* __restrict__ tw)
{
  fft_run<LOGN, CI, SPLIT>(v, i, reg, i, reg, lds, tw);
}

// The same transform with each thread holding TWO positions of one transform (32 points: virtual
// threads ia and ib = ia + T/2 of region reg), so half as many threads cover the workgroup's
// transforms and each has twice the registers. Radix-16 stages only (N = 16^k); CI > 0 layouts,
// split exchanges. Both groups are written before the barrier and read after it, so an exchange
// costs the same barriers as fft_run's.
template <int LOGN, int CI>
__device__ __forceinline__ void exchange_x2(CPair* va, CPair* vb, int reg, void* lds_raw, int ia, int ib, int base_a,
                                            int base_b, int st)
{
  using S = FftShape<LOGN>;
  float2* lds = reinterpret_cast<float2*>(lds_raw);
#pragma unroll
  for (int half = 0; half < 2; half++)
  {
#pragma unroll
    for (int t = 0; t < 16; t++)
    {
      lds[lds_slot<CI, S::PADDED>(reg, base_a + t * st)] = half_of(va[t], half);
      lds[lds_slot<CI, S::PADDED>(reg, base_b + t * st)] = half_of(vb[t], half);
    }
    XSYNC();
#pragma unroll
    for (int m = 0; m < 16; m++)
    {
      set_half(va[m], half, lds[lds_slot<CI, S::PADDED>(reg, read_pidx<LOGN>(ia, m))]);
      set_half(vb[m], half, lds[lds_slot<CI, S::PADDED>(reg, read_pidx<LOGN>(ib, m))]);
    }
    XSYNC();
  }
}

template <int LOGN, int CI>
__device__ __forceinline__ void fft_run_x2(CPair* va, CPair* vb, int ia, int reg, void* lds, const float2* __restrict__ tw)
{
  using S = FftShape<LOGN>;
  constexpr int N = S::N, T = S::T;
  static_assert(S::R0 == 16 && CI > 0, "radix-16 stages, column layout");
  const int ib = ia + T / 2;
  idft16(va);
  idft16(vb);
  // stage 0 outputs y[16 b + t] at pad16 = 17 b + t
  exchange_x2<LOGN, CI>(va, vb, reg, lds, ia, ib, 17 * ia, 17 * ib, 1);
  int p = 16;
#pragma unroll
  for (int s = 1; s < S::NSTAGE; s++)
  {
    const int stride = N / (16 * p);
    apply_stage_twiddles<LOGN>(va, (ia & (p - 1)) * stride, tw);
    apply_stage_twiddles<LOGN>(vb, (ib & (p - 1)) * stride, tw);
    idft16(va);
    idft16(vb);
    if (s + 1 < S::NSTAGE)
    {
      const int ja = (ia / p) * 16 * p + (ia & (p - 1)), jb = (ib / p) * 16 * p + (ib & (p - 1));
      exchange_x2<LOGN, CI>(va, vb, reg, lds, ia, ib, pad16(ja), pad16(jb), p + p / 16);
    }
    p *= 16;
  }
}

template <int LOGN>
__device__ __forceinline__ void load_twiddles(float2* tw_lds, const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  for (int e = threadIdx.x; e < S::TW_ENTRIES; e += blockDim.x)
    tw_lds[e] = tw_glob[e];
  __syncthreads();
}

}  // namespace oceanfft
