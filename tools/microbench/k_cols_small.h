// tools/microbench/k_cols_small.h (round 6, measured and not kept: DESIGN.md §4) — the half-spectrum column pass for whole grids that fill only part of the GPU
// (N = 1024 / 2048 with one or two cascades; BASELINE config 3 is one cascade of 2048^2): the same
// evolve (resources/spectrum.compute:183-240) and y iFFT of the five Hermitian field multiples of H as
// k_cols_half (device/k_half_cols.h), with EIGHT points per thread instead of sixteen.
//
// Why: k_cols_half holds 16 points per thread, so one 2048^2 cascade (257 strips of 4 columns) is
// 257 workgroups of 512 threads: 8 of a CU's 16 wave slots, one item each, and the pass is that one
// item's latency. With 8 points per thread the same strip is a 1024-thread workgroup (N / 8 threads
// per column): every wave slot of 257 CUs busy, half the serial work per thread. H of the thread's 8
// texels stays in VGPRs across the three field rounds (no H scratch). The transform is a radix-8
// Stockham FFT (fft8_run): a different radix split from fft_run's 16 x 16 x 8, so the fields differ
// from k_cols_half's in the last bits (FFT rounding, within the parity tolerances); the field layout
// (row groups RG / RGC, 4-column strips) and the Nyquist-row term are the same, so the production
// row pass reads them unchanged.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ocean_internal.h"
#include "device/evolve.h"
#include "device/fft.h"
#include "device/grid.h"
#include "device/memory.h"
#include "device/spectrum.h"
#include "device/k_half_cols.h"

namespace oceanfft
{

// Radix-8 Stockham shape: T = N / 8 threads per transform, thread i holding v[m] = x[i + m T]; a first
// stage of radix R0 = 2^(log2 N mod 3) (8 when it is 0) with span 1, then radix-8 stages; after the
// last one thread i holds X[i + m T] (self-sorting). tools/fft8_model.py plays the index arithmetic
// against N * ifft (tests/test_host_logic.py::test_fft8_index_model).
template <int LOGN>
struct Fft8Shape
{
  static constexpr int N = 1 << LOGN;
  static constexpr int T = N >> 3;
  static constexpr int LOG_R0 = (LOGN % 3) ? (LOGN % 3) : 3;
  static constexpr int R0 = 1 << LOG_R0;
  static constexpr int NSTAGE = 1 + (LOGN - LOG_R0) / 3;
  static constexpr int PADDED = N + N / 16;  // one pad slot per 16 elements, as fft.h
};

// v[t] *= w^t, t = 1..7, w = exp(+2 pi i e1 / N): w and w^4 from the exact table, the rest products
template <int LOGN>
__device__ __forceinline__ void apply_stage_twiddles8(CPair* v, int e1, const float2* __restrict__ tw)
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
}

// Write the 8 stage outputs at padded positions wp(t), barrier, read the next stage's inputs
// x[i + m T], barrier; split: one complex lane (float2) at a time, CI transforms interleaved.
template <int LOGN, int CI, typename WP>
__device__ __forceinline__ void exchange8(CPair* v, int reg, int i, void* lds_raw, WP wp)
{
  using S = Fft8Shape<LOGN>;
  float2* lds = reinterpret_cast<float2*>(lds_raw);
#pragma unroll
  for (int half = 0; half < 2; half++)
  {
#pragma unroll
    for (int t = 0; t < 8; t++)
      lds[lds_slot<CI, S::PADDED>(reg, wp(t))] = half_of(v[t], half);
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 8; m++)
      set_half(v[m], half, lds[lds_slot<CI, S::PADDED>(reg, pad16(i + m * S::T))]);
    __syncthreads();
  }
}

template <int LOGN, int CI>
__device__ __forceinline__ void fft8_run(CPair* v, int i, int reg, void* lds, const float2* __restrict__ tw)
{
  using S = Fft8Shape<LOGN>;
  constexpr int N = S::N, T = S::T, R0 = S::R0;
  if constexpr (R0 == 8)
  {
    idft8(v);
    if constexpr (S::NSTAGE > 1)
      exchange8<LOGN, CI>(v, reg, i, lds, [&](int t) { return pad16(8 * i + t); });
  }
  else
  {
    constexpr int U = 8 / R0;  // butterflies per thread; butterfly u = i + u T uses v[u + t U]
#pragma unroll
    for (int u = 0; u < U; u++)
    {
      CPair w[R0];
#pragma unroll
      for (int t = 0; t < R0; t++)
        w[t] = v[u + t * U];
      if constexpr (R0 == 2)
        idft2(w[0], w[1]);
      else
        idft4(w[0], w[1], w[2], w[3]);
#pragma unroll
      for (int t = 0; t < R0; t++)
        v[u + t * U] = w[t];
    }
    exchange8<LOGN, CI>(v, reg, i, lds, [&](int q) {
      const int u = q % U, t = q / U;
      return pad16((i + u * T) * R0 + t);
    });
  }
  int p = R0;
#pragma unroll
  for (int s = 1; s < S::NSTAGE; s++)
  {
    const int k = i & (p - 1);
    apply_stage_twiddles8<LOGN>(v, k * (N / (8 * p)), tw);
    idft8(v);
    if (s + 1 < S::NSTAGE)
    {
      const int j = (i / p) * 8 * p + k;
      const int pp = p;
      exchange8<LOGN, CI>(v, reg, i, lds, [&](int t) { return pad16(j + t * pp); });
    }
    p *= 8;
  }
}

template <int LOGN>
struct ColsSmallCfg
{
  static constexpr int B = 4;  // the whole-grid h0 / field strip width (HalfCfg<LOGN>::B)
  static constexpr int WG = Fft8Shape<LOGN>::T * B;
  static constexpr int LDS = ((FftShape<LOGN>::TW_ENTRIES * 8 + 15) / 16) * 16 + B * Fft8Shape<LOGN>::PADDED * 8;
};

// One item = one strip of 4 kept columns (u >= 0, or the Nyquist strip) of one cascade; thread (i, b)
// = column b, positions i + m T (m < 8). h0 is read once per texel (streamed) and H kept in VGPRs for
// the three field rounds (A, B), (D, E), (C, 0), stored as gab, gde, gc in k_cols_half's row-group
// layout. The workgroup of the last grid slot also writes the frame's Nyquist-row term into `spec`
// (half_nyquist_texel, as k_cols_half NYQ).
template <int LOGN, int RG, int RGC>
__global__ __launch_bounds__(ColsSmallCfg<LOGN>::WG, 4) void k_cols_small(FrameParams fp, const float4* __restrict__ h0,
                                                                          float4* __restrict__ gab,
                                                                          float4* __restrict__ gde,
                                                                          float2* __restrict__ gc,
                                                                          const float2* __restrict__ tw_glob,
                                                                          float4* __restrict__ spec)
{
  using S8 = Fft8Shape<LOGN>;
  using HC = HalfCfg<LOGN>;
  constexpr int N = S8::N, T = S8::T, B = ColsSmallCfg<LOGN>::B, STRIPS = HC::STRIPS, WG = ColsSmallCfg<LOGN>::WG;
  static_assert(HC::B == B && HC::SUPPORTED, "whole-grid half path, 4-column strips");
  static_assert(T % RG == 0 && T % RGC == 0, "a thread's rows i + m T stay in its row group's position");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((FftShape<LOGN>::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);
  const float dim = (float)N;
  const int total = fp.cascades * STRIPS;
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    const int c = item / STRIPS, s = item - c * STRIPS;
    const int t = opaque((int)threadIdx.x);
    const int b = t % B, i = t / B;
    const int xb = s == STRIPS - 1 ? 0 : N / (2 * B) + s;  // u >= 0 at x = N/2 + u; the Nyquist strip x = 0..3
    const int x = xb * B + b;
    const CascadeFrame f = fp.c[c];
    const float4* src = h0 + ((size_t)c * (N / B) + xb) * N * B;
    float2 H[8];
    {
      const int voff = (i * B + b) * 16;
      float4 a[8];
#pragma unroll
      for (int m = 0; m < 8; m++)  // fftShift on y folded into the load: input i + m T sits in row i + ((m + 4) mod 8) T
        a[m] = ld4s<kStream>(src, voff, ((m + 4) & 7) * T * B * 16);
#pragma unroll
      for (int m = 0; m < 8; m++)
      {
        const int y = i + ((m + 4) & 7) * T;
        H[m] = evolve(a[m], make_kvec(x, y, dim, f.dk).k, f);
      }
    }
    const size_t gbase = (size_t)c * STRIPS * N * B + half_group_offset<LOGN, RG>(0, s);
    const size_t cgbase = (size_t)c * STRIPS * N * B + half_group_offset<LOGN, RGC>(0, s);
#pragma unroll
    for (int round = 0; round < 3; round++)
    {
      CPair v[8];
#pragma unroll
      for (int m = 0; m < 8; m++)
      {
        const int y = i + ((m + 4) & 7) * T;
        const KVec q = make_kvec(x, y, dim, f.dk);
        const float2 h = H[m];
        if (round == 0)  // (A, B) = (H, kz H)
          v[m] = CPair{f2v{h.x, q.kz * h.x}, f2v{h.y, q.kz * h.y}};
        else if (round == 1)  // (D, E) = (kz H / |k|, kz^2 H / |k|)
        {
          const float e = q.kz * q.dirz;
          v[m] = CPair{f2v{q.dirz * h.x, e * h.x}, f2v{q.dirz * h.y, e * h.y}};
        }
        else  // (C, 0) = (H / |k|, 0)
          v[m] = CPair{f2v{q.inv * h.x, 0.0f}, f2v{q.inv * h.y, 0.0f}};
      }
      fft8_run<LOGN, B>(v, opaque(i), b, xch, tw);  // v[m] = field row i + m T
#pragma unroll
      for (int m = 0; m < 8; m++)
      {
        if (round == 0)
          st4s<kStream>(gab + gbase, half_group_offset<LOGN, RG>(i, 0, b) * 16, half_group_offset<LOGN, RG>(m * T, 0) * 16,
                        pair_raw(v[m]));
        else if (round == 1)
          st4s<kStream>(gde + gbase, half_group_offset<LOGN, RG>(i, 0, b) * 16, half_group_offset<LOGN, RG>(m * T, 0) * 16,
                        pair_raw(v[m]));
        else
          st2s<kStream>(gc + cgbase, half_group_offset<LOGN, RGC>(i, 0, b) * 8, half_group_offset<LOGN, RGC>(m * T, 0) * 8,
                        make_float2(v[m].re.x, v[m].im.x));
      }
    }
  }
  if ((int)blockIdx.x == (int)gridDim.x - 1)
    for (int idx = threadIdx.x; idx < fp.cascades * N; idx += WG)
      half_nyquist_texel(fp, N, B, h0, spec, nullptr, 1, 0, nullptr, nullptr, 0, idx);
}

}  // namespace oceanfft
