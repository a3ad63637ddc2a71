// device/k_rows_xs.h — the row pass of N = 16384 (the four-step path's blocks, RowSrc): one row of both
// images per 1024-thread workgroup with the x transform in four steps (XS, as k_rows_half<.., XS>),
// the next image's field loads in flight during the current image's transform (PF), and a streaming
// T_in (round 4): each kept element's own and -u CPairs are formed and their re-halves written to the
// LDS at once, only the im-halves wait in registers for the second half. 3.738 -> 3.680 ms per 16384^2
// pass (tools/microbench/rm16bench, profiles/r04_rm16bench_xs2.log; the round-3 form is k_rows_xs_r3
// in tools/microbench/ab_kernels.h; maps within 1e-7 of it, FMA contraction differs per kernel).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ocean_internal.h"
#include "device/fft.h"
#include "device/grid.h"
#include "device/k_half_rows.h"
#include "device/memory.h"

namespace oceanfft
{

// One row's 1024-thread workgroup holds 256 KiB of CPairs, half the CU's register file, so no second
// workgroup shares the CU and nothing else hides the loads: k_rows_half<.., XS> waits for each image's
// fields after the previous image's stores (3.81 ms per 16384^2 pass; 2.14 without loads,
// tools/microbench/rm16bench). PF issues the 16-B field loads of the NEXT image right after the
// current one's fields are consumed (image 1's (D, E) during image 0's transform; the next row's
// (A, B) during image 1's), so most of the HBM latency runs under the T_in / sub-transform / T_out
// phases. Registers: the 16 CPairs (64 VGPRs) and the prefetch (32); C (8 B per kept texel) is
// loaded where each image uses it (the second read of a row's C, ~20 us after the first, is served by
// L2): keeping it (16 VGPRs) beside the prefetch spills.
// EARLY (round 5): the next image's loads are issued before the current image's map stores instead
// of after them. A wave's vmcnt retires its memory instructions in issue order, so a load issued after
// 16 stores cannot be consumed before those stores are acknowledged: issued first, the next image's
// fields return while the current image's 256 KiB of stores drain. EARLY 1: image 1's 8 - PF field
// loads not already prefetched; 2: and its 8 C loads (held in 16 VGPRs until image 1's T_in); 3 (PF 0,
// persistent grids): also the next row's image-0 fields and C before image 1's stores, the first
// row's in a prologue; 4 (production): as 3, with image 0's C kept in those 16 VGPRs for image 1
// instead of re-read (no spills once nothing else is prefetched during the transform; the re-read
// missed L2 often enough to make the pass read 1.087 x its bytes): 3.144 -> 3.076 ms, same box,
// bit-identical (profiles/r05_rm16bench_keepc.log). rm16bench (profiles/r05_rm16bench_early.log, one box): PF 2 (round 4) 3.586 ms,
// EARLY 1 3.467 (PF 2) / 3.596 (PF 0), EARLY 2 3.336 / 3.330, maps bit-identical. Measured and not kept:
// also image 1's spec texels or its Nyquist texel before the stores (50-110 VGPRs spilled, 4.3-4.9
// ms; the Nyquist texel beside EARLY 3 still spills 69, 4.27 ms, profiles/r05_rm16bench_early_nyq.log);
// without image 1's spec loads at all (a timing ablation) EARLY 2 gains only 1 % more.
template <int LOGN, int PF, int EARLY = 0>
__global__ __launch_bounds__(1024) void k_rows_xs(FrameParams fp, const float4* __restrict__ spec, float4* __restrict__ maps,
                                                   float* __restrict__ jac, FoamParams foam,
                                                   const float2* __restrict__ tw_glob, int rows, RowSrc rs,
                                                   const float2* __restrict__ tw2_glob)
{
  using S = FftShape<LOGN>;
  using X = XsCfg<LOGN>;
  constexpr int N = S::N, T = S::T, L2 = X::L2, RS = X::RS;
  static_assert(T == 1024, "one 16-wave row per workgroup");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  float2* tw2 = reinterpret_cast<float2*>(smem + X::TW1);
  float2* xs = reinterpret_cast<float2*>(smem + X::TW1 + X::TW2);
  for (int e = threadIdx.x; e < FftShape<L2>::TW_ENTRIES; e += blockDim.x)
    tw2[e] = tw2_glob[e];
  load_twiddles<LOGN>(tw, tw_glob);

  const int total = fp.cascades * rows;
  const float dim = (float)N;
  // Element u = m T + i of a row sits in source block u >> log2(cpr) (RowSrc: each block holds cpr
  // columns of every row). A wave's 64 lanes cover 64 consecutive u inside one block (cpr is a
  // multiple of 64), so the block index is wave-uniform: it is computed from the wave's first thread
  // (readfirstlane, kept in SGPRs by sopaque) with a shift, and each load is one buffer descriptor for
  // the wave plus a lane offset.
  const int lcpr = 31 - __builtin_clz(rs.cpr), cmask = rs.cpr - 1;
  const int wave0 = __builtin_amdgcn_readfirstlane((int)threadIdx.x & ~63);
  static_assert(EARLY < 3 || PF == 0, "EARLY 3 carries the fields itself");
  float4 fp4[8], nx4[8];
  float2 ccn[EARLY >= 2 ? 8 : 1];  // EARLY 2+: the next image's C, loaded before the current image's stores
  auto issue_c = [&](int item, float2* cp) __attribute__((always_inline)) {
    const int c = item / rows, yl = item - c * rows;
    const size_t base = ((size_t)c * rows + yl) * rs.lp;
    const int i = opaque((int)threadIdx.x);
#pragma unroll
    for (int m = 0; m < 8; m++)
    {
      const int src = (m * T + sopaque(wave0)) >> lcpr;
      cp[m] = ld2<0>(reinterpret_cast<const float2*>(rs.c + (size_t)src * rs.src_stride) + base, ((m * T + i) & cmask) * 8);
    }
  };
  auto issue = [&](int item, int img, float4* p4, int m0, int m1) __attribute__((always_inline)) {
    const int c = item / rows, yl = item - c * rows;
    const size_t base = ((size_t)c * rows + yl) * rs.lp;
    const int i = opaque((int)threadIdx.x);
#pragma unroll
    for (int m = m0; m < m1; m++)
    {
      const int src = (m * T + sopaque(wave0)) >> lcpr;
      const size_t sb = (size_t)src * rs.src_stride;
      p4[m] = ld4<kStream>(reinterpret_cast<const float4*>((img == 0 ? rs.ab : rs.de) + sb) + base,
                           ((m * T + i) & cmask) * 16);
    }
  };
  int item = blockIdx.x;
  if (PF > 0 && item < total)
    issue(item, 0, fp4, 0, PF);
  if (EARLY >= 3 && item < total)
  {
    issue(item, 0, fp4, 0, 8);
    issue_c(item, ccn);
  }
  for (; item < total; item += gridDim.x)
  {
    const int c = item / rows, yl = item - c * rows;
    const float dk = fp.c[c].dk;
    const float sgy = (yl & 1) ? -1.0f : 1.0f;
    const size_t base = ((size_t)c * rows + yl) * rs.lp;
#pragma unroll
    for (int img = 0; img < 2; img++)
    {
      const int cimg = c * 2 + img;
      const int tid = opaque((int)threadIdx.x), i = tid;
      const float4* sp = spec + (size_t)cimg * N;
      if (!(EARLY && img == 1) && EARLY < 3)  // EARLY: issued before the previous image's stores
        issue(item, img, fp4, PF, 8);
      auto pslot = [&](int n) { return (n & 15) * RS + (n >> 4); };
      // thread 0: the Nyquist column (u = -N/2) takes the -u lane of u = 0 (T_in slot N/2)
      CPair nyq{};
      if (i == 0)
      {
        const size_t ns = (size_t)rs.nyq_src * rs.src_stride;
        const float kx = -(dim / 2.0f) * dk;
        const float2 cc = ld2<kStream>(reinterpret_cast<const float2*>(rs.c + ns) + base, rs.cpr * 8);
        const float4 t = ld4<kStream>(reinterpret_cast<const float4*>((img == 0 ? rs.ab : rs.de) + ns) + base,
                                      rs.cpr * 16);
        const CPair p = raw_pair(t);
        if (img == 0)
          nyq = CPair{f2v{(1.0f - kx) * p.re.x, -p.im.y - kx * cc.x}, f2v{(1.0f - kx) * p.im.x, p.re.y - kx * cc.y}};
        else
        {
          const float kx2 = kx * kx;
          nyq = CPair{f2v{-(p.im.x - kx2 * cc.y), -p.re.y + kx * p.im.x}, f2v{p.re.x - kx2 * cc.x, -p.im.y - kx * p.re.x}};
        }
      }
      // T_in: the lanes at u and at -u of the reference's 4 packed fields are rebuilt from the kept
      // half (Hermitian symmetry + the Nyquist-row term (-1)^y spec) and scattered into
      // the LDS in the first step's order: element n of the row goes to slot pslot(n) = (n % 16) * RS
      // + n / 16, so sub-transform n1 = n % 16 reads its 1024 inputs from one contiguous region of RS
      // slots (RS = 1 mod 16 keeps 16-lane writes on distinct banks). The LDS holds one half (re or
      // im plane) of the CPairs at a time: the re-halves are written as each element is formed, the
      // im-halves wait in ho / hn until the first half has been read back.
      __syncthreads();  // the previous image's T_out reads are done: T_in's first half streams in now
      float2 ho[8], hn[8];  // the im halves of the own and -u lanes, written after the first half
#pragma unroll
      for (int m = 0; m < 8; m++)
      {
        const int u = m * T + i;
        const float kx = (float)u * dk;
        const float4 s4 = ld4<0>(sp, (N / 2 - u) * 16);
        const int src = (m * T + sopaque(wave0)) >> lcpr;
        const float2 cc = (EARLY >= 2 && img == 1) || EARLY >= 3
                              ? ccn[m]
                              : ld2<0>(reinterpret_cast<const float2*>(rs.c + (size_t)src * rs.src_stride) + base,
                                       (u & cmask) * 8);
        CPair own, neg;
        if (img == 0)
        {
          const CPair p = raw_pair(fp4[m]);
          const float Ar = p.re.x, Ai = p.im.x, Br = p.re.y, Bi = p.im.y, Cr = cc.x, Ci = cc.y;
          own = CPair{f2v{(1.0f - kx) * Ar, -Bi - kx * Cr}, f2v{(1.0f - kx) * Ai, Br - kx * Ci}};
          neg = CPair{f2v{(1.0f + kx) * Ar + sgy * s4.x, -Bi + kx * Cr + sgy * s4.z},
                      f2v{-(1.0f + kx) * Ai + sgy * s4.y, -Br - kx * Ci + sgy * s4.w}};
        }
        else
        {
          const CPair q = raw_pair(fp4[m]);
          const float Cr = cc.x, Ci = cc.y, Dr = q.re.x, Di = q.im.x, Er = q.re.y, Ei = q.im.y;
          const float kx2 = kx * kx;
          own = CPair{f2v{-(Di - kx2 * Ci), -Er + kx * Di}, f2v{Dr - kx2 * Cr, -Ei - kx * Dr}};
          neg = CPair{f2v{-(Di + kx2 * Ci) + sgy * s4.x, -Er - kx * Di + sgy * s4.z},
                      f2v{-Dr - kx2 * Cr + sgy * s4.y, Ei - kx * Dr + sgy * s4.w}};
        }
        if (m == 0 && i == 0)
          neg = nyq;
        xs[pslot(i + m * T)] = half_of(own, 0);
        xs[pslot(m == 0 && i == 0 ? N / 2 : N - i - m * T)] = half_of(neg, 0);
        ho[m] = half_of(own, 1);
        hn[m] = half_of(neg, 1);
      }
      if constexpr (PF > 0)
      {
        if (img == 0)
          issue(item, 1, nx4, 0, PF);
        else if (item + (int)gridDim.x < total)
          issue(item + gridDim.x, 0, nx4, 0, PF);
      }
      // four-step x transform: wave w holds sub-transform n1 = w's 16 x 64 elements (the 1024-point
      // transform of region w runs inside the wave's own LDS region, whose exchanges need no
      // workgroup barrier), then the twiddles W_N^(n1 k2), then T_out: the region-major layout is
      // transposed through the LDS so each thread holds the 16 points of one 16-point DFT
      const int w = tid >> 6, l = tid & 63;
      CPair v[16];
      __syncthreads();
#pragma unroll
      for (int m = 0; m < 16; m++)
        set_half(v[m], 0, xs[w * RS + l + 64 * m]);
      __syncthreads();
#pragma unroll
      for (int m = 0; m < 8; m++)
      {
        xs[pslot(i + m * T)] = ho[m];
        xs[pslot(m == 0 && i == 0 ? N / 2 : N - i - m * T)] = hn[m];
      }
      __syncthreads();
#pragma unroll
      for (int m = 0; m < 16; m++)
        set_half(v[m], 1, xs[w * RS + l + 64 * m]);
      fft_run<L2, 0, true, true>(v, l, 0, l, 0, xs + w * RS, tw2);
      const float2 base_w = twiddle<LOGN>(w * l, tw);
#pragma unroll
      for (int m = 0; m < 16; m++)
        v[m] = cmul(v[m], base_w);
      apply_stage_twiddles<LOGN>(v, 64 * w, tw);
#pragma unroll
      for (int h = 0; h < 2; h++)
      {
        if (h)
          __syncthreads();
#pragma unroll
        for (int m = 0; m < 16; m++)
          xs[w * RS + l + 64 * m] = half_of(v[m], h);
        __syncthreads();
#pragma unroll
        for (int n1 = 0; n1 < 16; n1++)
          set_half(v[n1], h, xs[n1 * RS + tid]);
      }
      idft16(v);
      if constexpr (EARLY > 0)
      {
        if (img == 0)
        {
          issue(item, 1, fp4, EARLY >= 3 ? 0 : PF, 8);  // fp4 is free: image 0's fields were consumed by T_in
          if constexpr (EARLY >= 2 && EARLY != 4)  // EARLY 4: image 1 reuses image 0's C (kept in ccn)
            issue_c(item, ccn);
        }
        else if constexpr (EARLY >= 3)
        {
          // unconditional (the last row re-reads its own image 0: a conditional load would keep the
          // consumed fp4 / ccn live through image 1's transform as the loop's other incoming value)
          const int nx = item + (int)gridDim.x < total ? item + (int)gridDim.x : item;
          issue(nx, 0, fp4, 0, 8);
          issue_c(nx, ccn);
        }
      }
      float4* dst = maps + ((size_t)cimg * rows + yl) * N;
#pragma unroll
      for (int m = 0; m < 16; m++)
        st4<kStream>(dst + m * T, tid * 16, from_pair(v[m]));
      if (img == 1)
      {
        // computeFoam (resources/spectrum.compute:246-259): J = (1 + l dDx/dx)(1 + l dDz/dz) - l^2 (dDx/dz)^2
        // from the displacement map's .y, .z, .w, l = the cascade's displacement
        const float lam = foam.displacement[c];
        float* jb = jac + ((size_t)c * rows + yl) * N;
#pragma unroll
        for (int m = 0; m < 16; m++)
          st1<kStream>(jb + m * T, tid * 4,
                       (1.0f + lam * v[m].im.x) * (1.0f + lam * v[m].re.y) - lam * lam * v[m].im.y * v[m].im.y);
      }
#pragma unroll
      for (int m = 0; m < PF; m++)
        fp4[m] = nx4[m];
    }
  }
}

}  // namespace oceanfft
