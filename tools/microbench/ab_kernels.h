// ab_kernels.h — microbenchmark-only kernel variants and launchers (tools/microbench): the A/B
// alternatives measured against the production frame passes (DESIGN.md §4 "Tried and not kept",
// profiles/r0*_halfbench_*.log), kept out of liboceanfft.so. Production launchers: launch_half.hip,
// launch_slab.hip, launch_fft.hip. Included after them by all_kernels.h.
#pragma once

namespace oceanfft
{

// Pass 1 on half strips (whole grids): a 2T-thread workgroup (512 at N = 4096, 256 VGPRs, one per
// CU) transforms 2 columns per item, so the thread's 16 evolved amplitudes H stay in VGPRs (32)
// across the three rounds: no H scratch (k_cols_half<HS> moves 24 B per kept texel through it).
// Field strips are FB = 2 columns wide (half_group_offset<.., 2>): with RG rows per group, one store
// instruction of a wave (32 rows x 2 columns) writes whole 128-B lines when RG * 2 * 16 B = 128 B
// (gab, gde: RG = 4; gc: RGC = 8). The two halves of an h0 strip (items 2p, 2p + 1) run together
// on one XCD (xcd_pair_slot), so each 64-B h0 row is fetched once for both (default-policy loads).
// The Nyquist strip's second half (columns 2, 3: u < 0) is not needed and is skipped. The exchange
// moves whole CPairs (2 x PADDED x 16 B = 139 KiB of LDS at N = 4096).
// A/B only (launch_half_columns variants 12..14 with launch_half_rows 12..14; halfbench,
// profiles/r01_halfbench_halfstrips.log): pass 1 takes 0.81 ms against 0.96, but pass 2 then reads
// half lines (a 2-row item holds half of each 4-row x 2-column line): 1.64 ms against 1.52, frame
// 2.447 against 2.486 ms. Half-line stores (RG = 2, paired workgroups, default policy) lose the pass-1
// gain instead (0.96 ms). Production keeps 4-column items with the H scratch.
// The field CPair of a round: (A, B), (D, E) or (C, 0) from H (k_cols_half's pack).
template <int LOGN>
__device__ __forceinline__ CPair half_round_pack(int round, float2 H, const KVec& q)
{
  if (round == 0)  // (A, B) = (H, kz H)
    return CPair{f2v{H.x, q.kz * H.x}, f2v{H.y, q.kz * H.y}};
  if (round == 1)  // (D, E) = (kz H / |k|, kz^2 H / |k|)
  {
    const float e = q.kz * q.dirz;
    return CPair{f2v{q.dirz * H.x, e * H.x}, f2v{q.dirz * H.y, e * H.y}};
  }
  return CPair{f2v{q.inv * H.x, 0.0f}, f2v{q.inv * H.y, 0.0f}};  // (C, 0) = (H / |k|, 0)
}

// SAC: gc's store policy (default: SA).
template <int LOGN, int LA = 0, int SA = kStream, int RG = 4, int RGC = 8, int SAC = SA>
__global__ __launch_bounds__(2 * FftShape<LOGN>::T) void k_cols_half2(FrameParams fp, const float4* __restrict__ h0,
                                                                      float4* __restrict__ gab, float4* __restrict__ gde,
                                                                      float2* __restrict__ gc,
                                                                      const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  using K = ColFirstCfg<LOGN>;
  using HC = HalfCfg<LOGN>;
  constexpr int N = S::N, T = S::T, B = K::B, STRIPS = HC::STRIPS, FS = 2 * STRIPS;
  static_assert(HC::SUPPORTED && B == 4, "half strips of 4-column h0 strips");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);

  const int total = fp.cascades * FS;
  const float dim = (float)N;
  for (int item = xcd_pair_slot(blockIdx.x, gridDim.x); item < total; item += gridDim.x)
  {
    const int c = item / FS, fs = item - c * FS, s = fs >> 1, h = fs & 1;
    if (s == STRIPS - 1 && h == 1)
      continue;  // Nyquist strip, columns 2 and 3 (u < 0): unused (uniform per workgroup)
    const int xb = s == STRIPS - 1 ? 0 : N / (2 * B) + s;
    const CascadeFrame f = fp.c[c];
    const float4* src = h0 + ((size_t)c * (N / B) + xb) * N * B;
    const size_t cbase = (size_t)c * STRIPS * N * B;
    const size_t gbase = cbase + half_group_offset<LOGN, RG, 2>(0, fs);
    const size_t cgbase = cbase + half_group_offset<LOGN, RGC, 2>(0, fs);
    float2 H[16];
    {
      const int tid = opaque((int)threadIdx.x);
      const int b2 = tid % 2, i = (tid / 2) % T, x = xb * B + 2 * h + b2;
      const int voff = (i * B + 2 * h + b2) * 16;
      float4 a[16];
#pragma unroll
      for (int m = 0; m < 16; m++)  // fftShift on y folded into the load
        a[m] = ld4<LA>(src + ((m + 8) & 15) * T * B, voff);
#pragma unroll
      for (int m = 0; m < 16; m++)
      {
        const int y = i + ((m + 8) & 15) * T;
        H[m] = evolve(a[m], make_kvec(x, y, dim, f.dk).k, f);
      }
    }
#pragma unroll
    for (int round = 0; round < 3; round++)
    {
      // k-vectors recomputed per round (opaque: CSE would keep 48 of them live)
      const int tr = opaque((int)threadIdx.x);
      const int br = tr % 2, ir = (tr / 2) % T, xr = xb * B + 2 * h + br;
      CPair v[16];
#pragma unroll
      for (int m = 0; m < 16; m++)
      {
        const int y = ir + ((m + 8) & 15) * T;
        v[m] = half_round_pack<LOGN>(round, H[m], make_kvec(xr, y, dim, f.dk));
      }
      fft_run<LOGN, 2, false>(v, ir, br, xch, tw);
#pragma unroll
      for (int m = 0; m < 16; m++)
      {
        if (round == 0)
          st4<SA>(gab + gbase + half_group_offset<LOGN, RG, 2>(m * T, 0), half_group_offset<LOGN, RG, 2>(ir, 0, br) * 16,
                  pair_raw(v[m]));
        else if (round == 1)
          st4<SA>(gde + gbase + half_group_offset<LOGN, RG, 2>(m * T, 0), half_group_offset<LOGN, RG, 2>(ir, 0, br) * 16,
                  pair_raw(v[m]));
        else
          st2<SAC>(gc + cgbase + half_group_offset<LOGN, RGC, 2>(m * T, 0), half_group_offset<LOGN, RGC, 2>(ir, 0, br) * 8,
                  make_float2(v[m].re.x, v[m].im.x));
      }
    }
  }
}

// Pass 1 with H in VGPRs (whole grids, N = 4096): one 4-column strip per item on T * B / 2 = 512
// threads, each holding two positions (ia, ia + T/2) of one column, i.e. 32 points (fft_run_x2), so
// the 32 evolved amplitudes H (64 VGPRs) stay in registers across the three rounds: no H scratch
// (k_cols_half<HS> moves 24 B per kept texel through it) and h0 read once. Each store instruction of
// a wave still covers 16 rows x 4 columns, i.e. whole 128-B lines of the row-group layout. 512
// threads with 139 KiB of LDS: one workgroup per CU, 256 VGPRs per thread.
// HB: the second position's H goes through a per-block scratch slice (hs) instead (fewer VGPRs).
template <int LOGN, int LA = kStream, int SA = kStream, int RG = kHalfRG, int RGC = kHalfRGC, bool HB = false>
__global__ __launch_bounds__(FftShape<LOGN>::T * 2) void k_cols_half4(FrameParams fp, const float4* __restrict__ h0,
                                                                      float4* __restrict__ gab, float4* __restrict__ gde,
                                                                      float2* __restrict__ gc,
                                                                      const float2* __restrict__ tw_glob,
                                                                      float2* __restrict__ hs)
{
  using S = FftShape<LOGN>;
  using K = ColFirstCfg<LOGN>;
  using HC = HalfCfg<LOGN>;
  constexpr int N = S::N, T = S::T, B = K::B, STRIPS = HC::STRIPS;
  static_assert(HC::SUPPORTED && B == 4 && S::R0 == 16, "4-column strips, radix-16 stages");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);
  const int total = fp.cascades * STRIPS;
  const float dim = (float)N;
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    const int c = item / STRIPS, s = item - c * STRIPS;
    const int xb = s == STRIPS - 1 ? 0 : N / (2 * B) + s;
    const CascadeFrame f = fp.c[c];
    const float4* src = h0 + ((size_t)c * (N / B) + xb) * N * B;
    const size_t gbase = (size_t)c * STRIPS * N * B + half_group_offset<LOGN, RG>(0, s);
    const size_t cgbase = (size_t)c * STRIPS * N * B + half_group_offset<LOGN, RGC>(0, s);
    float2 H[HB ? 1 : 2][16];
    float2* hsb = hs + (size_t)blockIdx.x * 16 * (T * 2);
    {
      const int tid = opaque((int)threadIdx.x);
      const int b = tid % B, ia = (tid / B) % (T / 2), x = xb * B + b;
#pragma unroll
      for (int g = 0; g < 2; g++)
      {
        const int p = ia + g * (T / 2);
        float4 a[16];
#pragma unroll
        for (int m = 0; m < 16; m++)  // fftShift on y folded into the load
          a[m] = ld4s<LA>(src, (p * B + b) * 16, ((m + 8) & 15) * T * B * 16);
#pragma unroll
        for (int m = 0; m < 16; m++)
        {
          const float2 h = evolve(a[m], make_kvec(x, p + ((m + 8) & 15) * T, dim, f.dk).k, f);
          if (HB && g == 1)
            st2s<0>(hsb, tid * 8, m * (T * 2) * 8, h);
          else
            H[g][m] = h;
        }
      }
    }
#pragma unroll
    for (int round = 0; round < 3; round++)
    {
      // k-vectors recomputed per round (opaque: CSE would keep them live across the rounds)
      const int tid = opaque((int)threadIdx.x);
      const int b = tid % B, ia = (tid / B) % (T / 2), x = xb * B + b;
      CPair v[2][16];
#pragma unroll
      for (int g = 0; g < 2; g++)
#pragma unroll
        for (int m = 0; m < 16; m++)
        {
          const float2 h = (HB && g == 1) ? ld2s<kStream>(hsb, tid * 8, m * (T * 2) * 8) : H[g == 1 && HB ? 0 : g][m];
          v[g][m] = half_round_pack<LOGN>(round, h, make_kvec(x, ia + g * (T / 2) + ((m + 8) & 15) * T, dim, f.dk));
        }
      fft_run_x2<LOGN, B>(v[0], v[1], ia, b, xch, tw);
#pragma unroll
      for (int g = 0; g < 2; g++)
      {
        const int p = ia + g * (T / 2);
#pragma unroll
        for (int m = 0; m < 16; m++)
        {
          if (round == 0)
            st4s<SA>(gab + gbase, half_group_offset<LOGN, RG>(p, 0, b) * 16, half_group_offset<LOGN, RG>(m * T, 0) * 16,
                     pair_raw(v[g][m]));
          else if (round == 1)
            st4s<SA>(gde + gbase, half_group_offset<LOGN, RG>(p, 0, b) * 16, half_group_offset<LOGN, RG>(m * T, 0) * 16,
                     pair_raw(v[g][m]));
          else
            st2s<SA>(gc + cgbase, half_group_offset<LOGN, RGC>(p, 0, b) * 8, half_group_offset<LOGN, RGC>(m * T, 0) * 8,
                     make_float2(v[g][m].re.x, v[g][m].im.x));
        }
      }
    }
  }
}

// launch_half_columns with the A/B variants of halfbench (0 = production, numbered as in the logs)
hipError_t launch_half_columns_ab(int logn, const FrameParams& fp, const float4* h0, float4* gab, float4* gcd, float2* ge,
                               float4* spec, const float2* tw, hipStream_t stream, int cus, float2* hs = nullptr,
                               int hs_blocks = 0, const void* seed_consts = nullptr, int variant = 0)
{
  const SpectrumConsts* seed = static_cast<const SpectrumConsts*>(seed_consts);
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (!HalfCfg<LOGN>::SUPPORTED || LOGN < 10)  // the half path: N = 1024 .. 4096
      return hipErrorInvalidValue;
    else
    {
      using K = ColFirstCfg<LOGN>;
      using S = FftShape<LOGN>;
      const int n = S::N;
      hipError_t e = launch_half_nyquist(fp, n, K::B, h0, spec, nullptr, 1, 0, seed, stream, cus);
      if (e != hipSuccess)
        return e;
      // hs: per-block H scratch (half_hs_bytes): H evolved once instead of once per round
      if (seed && !hs)
        return hipErrorInvalidValue;
      // HS: h0 is read once per item, streamed (nt), which leaves the XCD's L2 to the H scratch
      // (0.972 -> 0.935 ms, tools/microbench/halfbench). variant (halfbench): 1 = default-policy h0
      // loads, 2 = sc1 field stores (dropped from L2: slower), 3 = sc1 + nt stores
      // 4..7: field layouts with row groups (RG, RGC) = (2, 2), (2, 4), (4, 4), (1, 1) (launch_half_rows 8..11)
      constexpr int RG = kHalfRG, RGC = kHalfRGC;
      // whole grids below 4096 keep 2 H pairs in VGPRs: 128 VGPRs, so two (2048) or four (1024)
      // workgroups fit a CU (with 4: 134-136 VGPRs, one fewer)
      constexpr int HKW = LOGN == 12 ? kHalfHK : 2;
      // HP (the H scratch in 16-B pairs): 0.921 -> 0.910 ms (halfbench hpair); variant 23: unpaired
      auto kern = seed && variant == 33 ? k_cols_half<LOGN, 0, kStream, true, false, true, RG, RGC, K::B, true>
                  : seed ? k_cols_half<LOGN, 0, kStream, true, false, true, RG, RGC, K::B, true, false, kHalfHL, kHalfHKSeed>
                       : !hs ? k_cols_half<LOGN, 0, kStream, false, false, false, RG, RGC>
                       : variant == 1 ? k_cols_half<LOGN, 0, kStream, true, false, false, RG, RGC>
                       : variant == 2 ? k_cols_half<LOGN, kStream, 16, true, false, false, RG, RGC>
                       : variant == 3 ? k_cols_half<LOGN, kStream, 18, true, false, false, RG, RGC>
                       : variant == 4 ? k_cols_half<LOGN, kStream, kStream, true, false, false, 2, 2>
                       : variant == 5 ? k_cols_half<LOGN, kStream, kStream, true, false, false, 2, 4>
                       : variant == 6 ? k_cols_half<LOGN, kStream, kStream, true, false, false, 4, 4>
                       : variant == 7 ? k_cols_half<LOGN, kStream, kStream, true, false, false, 1, 1>
                       : variant == 23 ? k_cols_half<LOGN, kStream, kStream, true, false, false, RG, RGC>
                       : variant == 24 ? k_cols_half<LOGN, kStream, kStream, true, false, false, RG, RGC, K::B, true, true>
                       : variant == 25 ? k_cols_half<LOGN, kStream, kStream, true, false, false, RG, RGC, K::B, true, false, 1, 0>
                       : variant == 26 ? k_cols_half<LOGN, kStream, kStream, true, false, false, RG, RGC, K::B, true, false, 1, 1>
                       : variant == 27 ? k_cols_half<LOGN, kStream, kStream, true, false, false, RG, RGC, K::B, true, false, 1, 2>
                       : variant == 28 ? k_cols_half<LOGN, kStream, kStream, true, false, false, RG, RGC, K::B, true, false, 0, 2>
                       : variant == 29 ? k_cols_half<LOGN, kStream, kStream, true, false, false, RG, RGC, K::B, true, false, 1, 3>
                       : variant == 30 ? k_cols_half<LOGN, kStream, kStream, true, false, false, RG, RGC, K::B, true, false, 1, 4>
                       : variant == 31 ? k_cols_half<LOGN, kStream, kStream, true, false, false, RG, RGC, K::B, true, false, 1, 5>
                       : variant == 32 ? k_cols_half<LOGN, kStream, kStream, true, false, false, RG, RGC, K::B, true>
                       : variant == 34 ? k_cols_half<LOGN, kStream, kStream, true, false, false, 2, 2, K::B, true, false, kHalfHL, kHalfHK>
                       : variant == 35 ? k_cols_half<LOGN, kStream, kStream, true, false, false, 4, 4, K::B, true, false, kHalfHL, kHalfHK>
                       : variant == 36 ? k_cols_half<LOGN, kStream, kStream, true, false, false, 1, 1, K::B, true, false, kHalfHL, kHalfHK>
                                      : k_cols_half<LOGN, kStream, kStream, true, false, false, RG, RGC, K::B, true, false, kHalfHL, HKW>;
      if (variant >= 12 && variant <= 14 && !seed)  // half-strip items (k_cols_half2): H in VGPRs
      {
        auto hk = variant == 12   ? k_cols_half2<LOGN, 0, kStream, 4, 8>
                  : variant == 13 ? k_cols_half2<LOGN, 0, 0, 2, 4>
                                  : k_cols_half2<LOGN, 0, kStream, 4, 4, 0>;
        const int hlds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + 2 * S::PADDED * 16;
        const int hg = persistent_grid(hk, 2 * S::T, hlds, fp.cascades * 2 * HalfCfg<LOGN>::STRIPS, cus);
        hipLaunchKernelGGL(hk, dim3(hg), dim3(2 * S::T), hlds, stream, fp, h0, gab, gcd, ge, tw);
        return hipGetLastError();
      }
      if constexpr (FftShape<LOGN>::R0 == 16)
      if (variant == 22 && !seed)  // H in VGPRs: 32 points per thread, 512 threads (k_cols_half4)
      {
        auto hk = hs ? k_cols_half4<LOGN, kStream, kStream, kHalfRG, kHalfRGC, true> : k_cols_half4<LOGN>;
        const int hlds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + K::LDS1;
        int hg = persistent_grid(hk, S::T * 2, hlds, fp.cascades * HalfCfg<LOGN>::STRIPS, cus);
        if (hs && hg > hs_blocks)
          hg = hs_blocks;
        hipLaunchKernelGGL(hk, dim3(hg), dim3(S::T * 2), hlds, stream, fp, h0, gab, gcd, ge, tw, hs);
        return hipGetLastError();
      }
      if (variant == 20 && hs && !seed)  // half-strip items, two workgroups per CU (HS slices of half size)
      {
        auto hk = k_cols_half<LOGN, 0, 0, true, false, false, RG, RGC, K::B / 2>;
        const int wg = S::T * (K::B / 2);
        const int hlds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + (K::B / 2) * S::PADDED * 8;
        int hg = persistent_grid(hk, wg, hlds, fp.cascades * HalfCfg<LOGN>::STRIPS * 2, cus);
        const int slices = hs_blocks * (K::WG1 / wg);
        if (hg > slices)
          hg = slices;
        hg &= ~15;  // xcd_pair_slot needs a multiple of 16 blocks
        if (hg < 16)
          return hipErrorInvalidValue;
        hipLaunchKernelGGL(hk, dim3(hg), dim3(wg), hlds, stream, fp, h0, gab, gcd, ge, tw, hs, HalfSlab{},
                           (unsigned char*)nullptr, 1, seed);
        return hipGetLastError();
      }
      // H pairs in LDS (HL): production kHalfHL; variants 25..31 as named in halfbench hkeep, 32 none
      // the chain above with HL = 0 (34..36: production's H pairs with the field layouts of 4, 6, 7)
      const bool named = (variant >= 1 && variant <= 7) || (variant >= 23 && variant <= 32);
      const int hl = seed ? (variant == 33 ? 0 : kHalfHL)
                     : !hs ? 0 : !named ? kHalfHL : (variant >= 25 && variant <= 31 && variant != 28) ? 1 : 0;
      const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + K::LDS1 + hl * K::WG1 * 16;
      int grid = persistent_grid(kern, K::WG1, lds, fp.cascades * HalfCfg<LOGN>::STRIPS, cus);
      // hs holds hs_blocks slices for 1024-thread workgroups (half_hs_bytes); a block uses 16 x WG1
      // entries, so below 4096 each slice serves 1024 / WG1 blocks (variant 37: one, as before)
      const int slices = variant == 37 ? hs_blocks : hs_blocks * (1024 / K::WG1);
      if (hs && grid > slices)
        grid = slices;
      if (grid < 1)
        return hipErrorInvalidValue;
      hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG1), lds, stream, fp, h0, gab, gcd, ge, tw, hs, HalfSlab{},
                         (unsigned char*)nullptr, 1, seed);  // gcd/ge: (D, E) / C
      return hipGetLastError();
    }
  });
}

hipError_t launch_half_rows_ab(int logn, const FrameParams& fp, const float4* gab, const float4* gcd, const float2* ge,
                            const float4* rcorr, float4* maps, float* jac, const FoamParams& foam, const float2* tw,
                            hipStream_t stream, int cus, int ablation = 0)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (!HalfCfg<LOGN>::SUPPORTED)
      return hipErrorInvalidValue;
    else
    {
      using K = ColFirstCfg<LOGN>;
      using S = FftShape<LOGN>;
      // ablation (tools/microbench; 1-3 on the production shape): 1 no HBM loads, 2 no x transform,
      // 3 no mirror exchange,
      // 4 / 5 ColFirstCfg's rows per workgroup (one 1024-thread workgroup per CU) / one row
      // 0 (production): one item per row block for both images (C loaded once); 6: one image per
      // item (C loaded by both items of a row block)
      constexpr int R4 = K::RPW2;
      // production at N = 4096: one row (both images) per 256-thread workgroup, four workgroups per
      // CU, the 4 rows of a gc line on one XCD (GRP 4): 1.407 -> 1.377 ms per 8 x 4096^2, maps
      // bit-identical (halfbench rowv 16); 17 = the two-row workgroups (production below 4096)
      constexpr bool ONE_ROW = LOGN == 12;
      const int rpw = ablation == 4 ? R4
                      : (ablation == 5 || ablation == 16 || ablation == 18 || ablation == 19 || (ablation == 0 && ONE_ROW)) ? 1
                                                                                                             : 2;
      const int per_item = (ablation <= 3 || ablation >= 7) ? 1 : 2;
      // production loads use the default policy: C's 128-B lines are shared by the paired items
      // (xcd_pair_slot) and streamed loads lost them before the partner's read (-5 %,
      // tools/microbench/halfbench); 7: streamed loads
      // 8..11: the field layouts of launch_half_columns' variants 4..7
      constexpr int RG = kHalfRG, RGC = kHalfRGC;
      // 16: one row (both images) per 256-thread workgroup, four per CU, rows of a gc line on one XCD
      auto kern = ablation == 0 && ONE_ROW ? k_rows_half<LOGN, 0, kStream, 0, 1, true, false, RG, RGC, 4, 4>
                  : ablation == 0 || ablation == 17 ? k_rows_half<LOGN, 0, kStream, 0, 2, true, false, RG, RGC>
                  : ablation == 16 ? k_rows_half<LOGN, 0, kStream, 0, 1, true, false, RG, RGC, 4, 4>
                  // 18 / 19: one row per 256-thread workgroup on the half-strip layouts of pass-1 variants
                  // 12 / 14 (FB 2: gab/gde RG 4; gc RGC 8 / 4), the 4 rows of a 128-B line on one XCD
                  : ablation == 18 ? k_rows_half<LOGN, 0, kStream, 0, 1, true, false, 4, 8, 2, 4>
                  : ablation == 19 ? k_rows_half<LOGN, 0, kStream, 0, 1, true, false, 4, 4, 2, 4>
                  : ablation == 8 ? k_rows_half<LOGN, 0, kStream, 0, 2, true, false, 2, 2>
                  : ablation == 9 ? k_rows_half<LOGN, 0, kStream, 0, 2, true, false, 2, 4>
                  : ablation == 10 ? k_rows_half<LOGN, 0, kStream, 0, 2, true, false, 4, 4>
                  : ablation == 11 ? k_rows_half<LOGN, 0, kStream, 0, 2, true, false, 1, 1>
                  : ablation == 12 ? k_rows_half<LOGN, 0, kStream, 0, 2, true, false, 4, 8, 2, 4>
                  : ablation == 13 ? k_rows_half<LOGN, 0, kStream, 0, 2, true, false, 2, 4, 2, 2>
                  : ablation == 14 ? k_rows_half<LOGN, 0, kStream, 0, 2, true, false, 4, 4, 2, 2>
                  : ablation == 15 ? k_rows_half<LOGN, 0, kStream, 0, 2, true, false, RG, RGC, 4, 2, false>
                  : ablation == 7 ? k_rows_half<LOGN, kStream, kStream, 0, 2, true, false, RG, RGC>
                  : ablation == 6 ? k_rows_half<LOGN, kStream, kStream, 0, 2, false, false, RG, RGC>
                  : ablation == 1 ? k_rows_half<LOGN, 0, kStream, 1, 2, true, false, RG, RGC>
                  : ablation == 2 ? k_rows_half<LOGN, 0, kStream, 2, 2, true, false, RG, RGC>
                  : ablation == 3 ? k_rows_half<LOGN, 0, kStream, 3, 2, true, false, RG, RGC>
                  : ablation == 4 ? k_rows_half<LOGN, kStream, kStream, 0, R4>
                                  : k_rows_half<LOGN, kStream, kStream, 0, 1>;
      const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + lds_row_slots<LOGN>(rpw) * 8;
      const int grid = persistent_grid(kern, S::T * rpw, lds, fp.cascades * per_item * (S::N / rpw), cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(S::T * rpw), lds, stream, fp, gab, gcd, ge, rcorr, maps, jac, foam, tw,
                         S::N, RowSrc{}, (const float2*)nullptr);
      return hipGetLastError();
    }
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

// Round 2's step 1 (whole grids only, compile-time pitch; its h0 descriptor per lane became a
// waterfall loop per load): the same-box reference for k_gen4_step1 (gen4bench)
template <int LOGN>
struct Gen4CfgR2
{
  static constexpr int N = 1 << LOGN, N2 = N / 16, B = ColFirstCfg<LOGN>::B, KP = N / 2 + B;
  static constexpr int PITCH = (KP + 15) / 16 * 16;
};

template <int LOGN, int MINW = 1>
__global__ __launch_bounds__(256, MINW) void k_gen4_step1_r2(FrameParams fp, const float4* __restrict__ h0,
                                                    unsigned char* __restrict__ parts, const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  using G = Gen4CfgR2<LOGN>;
  constexpr int N = G::N, N2 = G::N2, KP = G::KP, PITCH = G::PITCH, XB = (KP + 63) / 64;
  __shared__ float2 tw[S::TW_ENTRIES];
  load_twiddles<LOGN>(tw, tw_glob);
  const size_t part = (size_t)fp.cascades * N * PITCH;  // texels per part
  float4* gab = reinterpret_cast<float4*>(parts);
  float4* gde = gab + part;
  float2* gc = reinterpret_cast<float2*>(gde + part);
  const int total = fp.cascades * XB * (N2 / 4);
  const float dim = (float)N;
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int t = item;
    const int xbk = t % XB;
    t /= XB;
    const int n2 = (t % (N2 / 4)) * 4 + wv, c = t / (N2 / 4);
    const int u = xbk * 64 + lane;
    const bool live = u < KP;
    const int uc = live ? u : KP - 1;  // columns past the last: loads clamped, nothing stored
    const int x = uc < N / 2 ? N / 2 + uc : uc - N / 2;
    const CascadeFrame f = fp.c[c];
    // one descriptor for the item's h0 strip (uniform: 64 lanes = one 64-column block)
    const float4* src = h0 + ((size_t)c * (N / kGen4Block) + x / kGen4Block) * N * kGen4Block;
    const int loff = (n2 * kGen4Block + (x % kGen4Block)) * 16;
    float2 H[16];
    {
      float4 a[16];
#pragma unroll
      for (int n1 = 0; n1 < 16; n1++)
        a[n1] = ld4s<kStream>(src, loff, N2 * ((n1 + 8) & 15) * kGen4Block * 16);
#pragma unroll
      for (int n1 = 0; n1 < 16; n1++)
        H[n1] = evolve(a[n1], make_kvec(x, N2 * ((n1 + 8) & 15) + n2, dim, f.dk).k, f);
    }
    // output row N2 k1 + n2 of the cascade: two descriptors per part (k1 < 8, k1 >= 8) keep the
    // 32-bit offsets below 2 GiB
    const size_t cb = (size_t)c * N * PITCH;
    const int soff = (n2 * PITCH + u) * 16;
#pragma unroll
    for (int round = 0; round < 2; round++)
    {
      const int xr = opaque(x), n2r = opaque(n2);
      CPair v[16];
#pragma unroll
      for (int n1 = 0; n1 < 16; n1++)
      {
        const KVec q = make_kvec(xr, N2 * ((n1 + 8) & 15) + n2r, dim, f.dk);
        const float2 h = H[n1];
        if (round == 0)  // (A, B) = (H, kz H)
          v[n1] = CPair{f2v{h.x, q.kz * h.x}, f2v{h.y, q.kz * h.y}};
        else  // (D, E) = (kz H / |k|, kz^2 H / |k|)
        {
          const float e = q.kz * q.dirz;
          v[n1] = CPair{f2v{q.dirz * h.x, e * h.x}, f2v{q.dirz * h.y, e * h.y}};
        }
      }
      idft16(v);
      apply_stage_twiddles<LOGN>(v, n2r, tw);
      float4* d0 = (round == 0 ? gab : gde) + cb;
      float4* d1 = d0 + (size_t)8 * N2 * PITCH;
      if (live)
#pragma unroll
        for (int k1 = 0; k1 < 16; k1++)
          st4s<kStream>(k1 < 8 ? d0 : d1, soff, (k1 & 7) * N2 * PITCH * 16, pair_raw(v[k1]));
    }
    {
      const int xr = opaque(x), n2r = opaque(n2);
      float2 w[16];  // C = H / |k|, one complex lane
#pragma unroll
      for (int n1 = 0; n1 < 16; n1++)
      {
        const float inv = make_kvec(xr, N2 * ((n1 + 8) & 15) + n2r, dim, f.dk).inv;
        w[n1] = make_float2(inv * H[n1].x, inv * H[n1].y);
      }
      idft16(w);
      apply_stage_twiddles<LOGN>(w, n2r, tw);
      float2* d0 = gc + cb;
      if (live)
#pragma unroll
        for (int k1 = 0; k1 < 16; k1++)
          st2s<kStream>(d0, soff / 2, k1 * N2 * PITCH * 8, w[k1]);
    }
  }
}


// The in-place column pass with GROUP strips per XCD group (ifft4bench)
template <int GROUP>
hipError_t launch_cols_group(int logn, int n_images, float4* images, const float2* tw, hipStream_t stream, int cus)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    using K = ColCfg<LOGN>;
    int lds = lds_bytes_cols<LOGN>();
    auto kern = k_cols<LOGN, GROUP>;
    int grid = persistent_grid(kern, K::WG, lds, n_images * K::STRIPS, cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG), lds, stream, n_images, images, tw);
    return hipGetLastError();
  });
}

// Column-first EncodeIFFT at N = 8192 (B = 2: 32-B strided pieces, GROUP strips per XCD group) through a
// work image, then the blocked row pass (ifft4bench)
template <int GROUP, int GRPR = 1>
hipError_t launch_ifft_colfirst13(int n_images, float4* images, float4* work, const float2* tw, hipStream_t stream,
                                  int cus)
{
  constexpr int LOGN = 13;
  using K = ColFirstCfg<LOGN>;
  using S = FftShape<LOGN>;
  constexpr int tw_lds = tw_bytes<S::TW_ENTRIES>();
  auto ka = k_cols_to_blocks<LOGN, 0, GROUP>;
  const int grid = persistent_grid(ka, K::WG1, tw_lds + K::LDS1, n_images * (S::N / K::B), cus);
  hipLaunchKernelGGL(ka, dim3(grid), dim3(K::WG1), tw_lds + K::LDS1, stream, n_images, images, work, tw);
  auto kb = k_rows_final<LOGN, true, kStream, kStream, K::RPW2, 0, GRPR>;
  const SlabGeom g{0, S::N};
  const int grid2 = persistent_grid(kb, K::WG2, tw_lds + K::LDS2, n_images * (S::N / K::RPW2), cus);
  hipLaunchKernelGGL(kb, dim3(grid2), dim3(K::WG2), tw_lds + K::LDS2, stream, n_images, g, work, images,
                     (float*)nullptr, FoamParams{}, tw);
  return hipGetLastError();
}

// Column-first EncodeIFFT at any N (ifft4bench): the strided pass with GROUPC strips per XCD group
// (their partial-line reads meet in one L2), the blocked row pass with GRPR row items per XCD group
// RPW: rows per row-pass item (default ColFirstCfg's; 1 at 8192 halves the workgroup's LDS, so two
// workgroups share a CU)
template <int LOGN, int GROUPC, int GRPR, int RPW = ColFirstCfg<LOGN>::RPW2, int LAR = kStream>
hipError_t launch_ifft_colfirst_ab(int n_images, float4* images, float4* work, const float2* tw, hipStream_t stream,
                                   int cus)
{
  using K = ColFirstCfg<LOGN>;
  using S = FftShape<LOGN>;
  constexpr int tw_lds = tw_bytes<S::TW_ENTRIES>();
  constexpr int LDS2 = lds_row_slots<LOGN>(RPW) * 8;
  auto ka = k_cols_to_blocks<LOGN, 0, GROUPC>;
  const int grid = persistent_grid(ka, K::WG1, tw_lds + K::LDS1, n_images * (S::N / K::B), cus);
  hipLaunchKernelGGL(ka, dim3(grid), dim3(K::WG1), tw_lds + K::LDS1, stream, n_images, images, work, tw);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return e;
  auto kb = k_rows_final<LOGN, true, LAR, kStream, RPW, 0, GRPR>;
  const SlabGeom g{0, S::N};
  const int grid2 = persistent_grid(kb, S::T * RPW, tw_lds + LDS2, n_images * (S::N / RPW), cus);
  hipLaunchKernelGGL(kb, dim3(grid2), dim3(S::T * RPW), tw_lds + LDS2, stream, n_images, g, work, images,
                     (float*)nullptr, FoamParams{}, tw);
  return hipGetLastError();
}

// k_rows_xs before the scalar source-block shift (a division per field load): same-box A/B reference
// for rm16bench. Results are bit-identical to production's.
template <int LOGN, int PF>
__global__ __launch_bounds__(1024) void k_rows_xs_div(FrameParams fp, const float4* __restrict__ spec, float4* __restrict__ maps,
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
  // the 8 kept elements u = m T + tid of one image: (A, B) or (D, E)
  float4 fp4[8], nx4[8];
  auto issue = [&](int item, int img, float4* p4, int m0, int m1) __attribute__((always_inline)) {
    const int c = item / rows, yl = item - c * rows;
    const size_t base = ((size_t)c * rows + yl) * rs.lp;
    const int i = opaque((int)threadIdx.x);
#pragma unroll
    for (int m = m0; m < m1; m++)
    {
      const int u = m * T + i;
      const int src = __builtin_amdgcn_readfirstlane(u / rs.cpr);  // source block (wave-uniform)
      const int col = u - src * rs.cpr;
      const size_t sb = (size_t)src * rs.src_stride;
      p4[m] = ld4<kStream>(reinterpret_cast<const float4*>((img == 0 ? rs.ab : rs.de) + sb) + base, col * 16);
    }
  };
  int item = blockIdx.x;
  if (PF > 0 && item < total)
    issue(item, 0, fp4, 0, PF);
  for (; item < total; item += gridDim.x)
  {
    const int c = item / rows, yl = item - c * rows;
    const float dk = fp.c[c].dk;
    const float sgy = (yl & 1) ? -1.0f : 1.0f;  // (-1)^q of the Nyquist-row term (rows start at an even q)
    const size_t base = ((size_t)c * rows + yl) * rs.lp;
#pragma unroll
    for (int img = 0; img < 2; img++)
    {
      const int cimg = c * 2 + img;
      const int tid = opaque((int)threadIdx.x), i = tid;
      const float4* sp = spec + (size_t)cimg * N;
      issue(item, img, fp4, PF, 8);  // the elements not prefetched
      CPair v[16];  // own lanes in v[m], the -u lanes in v[m + 8] until the transposition
#pragma unroll
      for (int m = 0; m < 8; m++)
      {
        const int u = m * T + i;
        const float kx = (float)u * dk;
        const float4 s4 = ld4<0>(sp, (N / 2 - u) * 16);  // the -u column's Nyquist-row term (x = N/2 - u)
        const int src = __builtin_amdgcn_readfirstlane(u / rs.cpr);
        const float2 cc = ld2<0>(reinterpret_cast<const float2*>(rs.c + (size_t)src * rs.src_stride) + base,
                                 (u - src * rs.cpr) * 8);  // C
        if (img == 0)
        {
          const CPair p = raw_pair(fp4[m]);  // (A, B)
          const float Ar = p.re.x, Ai = p.im.x, Br = p.re.y, Bi = p.im.y, Cr = cc.x, Ci = cc.y;
          v[m] = CPair{f2v{(1.0f - kx) * Ar, -Bi - kx * Cr}, f2v{(1.0f - kx) * Ai, Br - kx * Ci}};
          v[m + 8] = CPair{f2v{(1.0f + kx) * Ar + sgy * s4.x, -Bi + kx * Cr + sgy * s4.z},
                           f2v{-(1.0f + kx) * Ai + sgy * s4.y, -Br - kx * Ci + sgy * s4.w}};
        }
        else
        {
          const CPair q = raw_pair(fp4[m]);  // (D, E)
          const float Cr = cc.x, Ci = cc.y, Dr = q.re.x, Di = q.im.x, Er = q.re.y, Ei = q.im.y;
          const float kx2 = kx * kx;
          v[m] = CPair{f2v{-(Di - kx2 * Ci), -Er + kx * Di}, f2v{Dr - kx2 * Cr, -Ei - kx * Dr}};
          v[m + 8] = CPair{f2v{-(Di + kx2 * Ci) + sgy * s4.x, -Er - kx * Di + sgy * s4.z},
                           f2v{-Dr - kx2 * Cr + sgy * s4.y, Ei - kx * Dr + sgy * s4.w}};
        }
      }
      if (i == 0)
      {
        // thread 0: the Nyquist column u = -N/2 (block nyq_src, column cpr) replaces the unused -u
        // lane of u = 0 (T_in puts v[8] at n = N/2)
        const size_t ns = (size_t)rs.nyq_src * rs.src_stride;
        const float kx = -(dim / 2.0f) * dk;
        const float2 cc = ld2<kStream>(reinterpret_cast<const float2*>(rs.c + ns) + base, rs.cpr * 8);
        const float4 t = ld4<kStream>(reinterpret_cast<const float4*>((img == 0 ? rs.ab : rs.de) + ns) + base,
                                      rs.cpr * 16);
        const CPair p = raw_pair(t);
        if (img == 0)
          v[8] = CPair{f2v{(1.0f - kx) * p.re.x, -p.im.y - kx * cc.x}, f2v{(1.0f - kx) * p.im.x, p.re.y - kx * cc.y}};
        else
        {
          const float kx2 = kx * kx;
          v[8] = CPair{f2v{-(p.im.x - kx2 * cc.y), -p.re.y + kx * p.im.x}, f2v{p.re.x - kx2 * cc.x, -p.im.y - kx * p.re.x}};
        }
      }
      // the next image's fields: this row's (D, E), or the next row's (A, B) and C
      if constexpr (PF > 0)
      {
        if (img == 0)
          issue(item, 1, nx4, 0, PF);
        else if (item + (int)gridDim.x < total)
          issue(item + gridDim.x, 0, nx4, 0, PF);
      }
      // x index n = n1 + 16 n2, output k = k2 + 1024 k1: T_in gives wave n1 = w the inputs x(w + 16 n2)
      // (own lanes at n, the -u lanes at N - n, thread 0's Nyquist column at N/2); the wave's
      // 1024-point sub-transform; times W_N^(n1 k2); T_out gives thread k2 = tid the 16 values
      // Z_n1(k2); the 16-point DFT over n1 leaves v[k1] = X(tid + T k1). LDS slot of n: (n mod 16) RS + n / 16.
      const int w = tid >> 6, l = tid & 63;
      auto pslot = [&](int n) { return (n & 15) * RS + (n >> 4); };
      __syncthreads();  // the previous image's T_out reads are done
#pragma unroll
      for (int h = 0; h < 2; h++)
      {
        if (h)
          __syncthreads();
#pragma unroll
        for (int m = 0; m < 8; m++)
        {
          xs[pslot(i + m * T)] = half_of(v[m], h);
          xs[pslot(m == 0 && i == 0 ? N / 2 : N - i - m * T)] = half_of(v[m + 8], h);
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < 16; m++)
          set_half(v[m], h, xs[w * RS + l + 64 * m]);
      }
      // region w is the wave's alone until T_out's first barrier: its exchanges need no barriers
      fft_run<L2, 0, true, true>(v, l, 0, l, 0, xs + w * RS, tw2);  // v[m] = Y_w(l + 64 m)
      const float2 base_w = twiddle<LOGN>(w * l, tw);
#pragma unroll
      for (int m = 0; m < 16; m++)
        v[m] = cmul(v[m], base_w);
      apply_stage_twiddles<LOGN>(v, 64 * w, tw);  // x W_N^(w (l + 64 m))
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
      float4* dst = maps + ((size_t)cimg * rows + yl) * N;
#pragma unroll
      for (int m = 0; m < 16; m++)
        st4<kStream>(dst + m * T, tid * 16, from_pair(v[m]));
      if (img == 1)
      {
        // displacementMap (Dz, dDx/dx, dDz/dz, dDx/dz) = (re0, im0, re1, im1): Jacobian,
        // spectrum.compute:246-259
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



// EncodeIFFT at 16384 with the radix-4 pre-stage on TWO columns per item and the residue pair
// (rp, rp + 2), which share their four loads: y_{rp} = s02 + w t13, y_{rp+2} = s02 - w t13 with
// s02 = x0 + (-1)^rp x2, t13 = x1 + (-1)^rp x3, w = i^rp (half the L2 reads per output of
// k_cols_pre<14>). Transform b4 = (column c = b4 & 1, s = b4 >> 1), residue r = rp + 2 s. Work
// layout [img][strip2][r][k'][2] (two 128-KiB runs per item); the row pass is k_rows_final with
// BO = 2, PR = 4 (32-B pieces, 4 stored rows per 128-B line on one XCD). prebench only.
template <int LA = 0>
__global__ __launch_bounds__(1024) void k_cols_pre_pair14(int images, const float4* __restrict__ src_images,
                                                          float4* __restrict__ work, const float2* __restrict__ twn_glob,
                                                          const float2* __restrict__ twm_glob)
{
  constexpr int LOGN = 14;
  using P = PreCfg;
  using SN = FftShape<LOGN>;
  constexpr int N = SN::N, M = P::M, R = 4, T = P::T, B = 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* twm = reinterpret_cast<float2*>(smem);
  float2* twn = reinterpret_cast<float2*>(smem + P::TWM);
  void* xch = smem + P::TWM + ((SN::TW_ENTRIES * 8 + 15) / 16) * 16;
  for (int e = threadIdx.x; e < SN::TW_ENTRIES; e += blockDim.x)
    twn[e] = twn_glob[e];
  load_twiddles<P::LOGM>(twm, twm_glob);
  const int strips = N / B;  // 2-column strips
  const int total = images * strips * 2;
  // item = ((img strips/4 + group) 2 + rp) 4 + strip & 3: the 8 items sharing lines are consecutive
  for (int item = xcd_group_slot<8>(blockIdx.x, gridDim.x); item < total; item += gridDim.x)
  {
    const int tid = opaque((int)threadIdx.x);
    const int b4 = tid & 3, i = tid >> 2, c = b4 & 1, s = b4 >> 1;
    const int it = __builtin_amdgcn_readfirstlane(item);
    int t = it >> 2;
    const int rp = t & 1;
    t >>= 1;
    const int grp = t % (strips / 4), img = t / (strips / 4);
    const int xb = grp * 4 + (it & 3);
    const int r = rp + 2 * s;  // per lane
    const float cs = rp ? -1.0f : 1.0f, sg = s ? -1.0f : 1.0f;
    const float2 w = make_float2(rp ? 0.0f : sg, rp ? sg : 0.0f);  // (-1)^s i^rp
    const float4* src = src_images + ((size_t)img << (2 * LOGN)) + (size_t)xb * B;
    const int voff = ((i << LOGN) + c) * 16;
    CPair v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
    {
      CPair x[R];
#pragma unroll
      for (int j = 0; j < R; j++)
      {
        const unsigned row = (unsigned)((m * T + j * M + N / 2) & (N - 1));
        x[j] = to_pair(ld4<LA>(src, (int)((unsigned)voff + (row << (LOGN + 4))), -1));
      }
      const f2v cc = {cs, cs};
      const CPair s02 = {x[0].re + cc * x[2].re, x[0].im + cc * x[2].im};
      const CPair t13 = {x[1].re + cc * x[3].re, x[1].im + cc * x[3].im};
      v[m] = cmul(s02 + cmul(t13, w), twiddle<LOGN>((i + m * T) * r, twn));
      if ((m & 1) == 1)
        asm volatile("" ::: "memory");
    }
    fft_run<P::LOGM, 4, true>(v, i, b4, xch, twm);  // v[m] = X[4 (i + m T) + r] of column c
    // run (xb, r) = (xb, rp) + 2 s runs: a wave-uniform base, the residue's run in the lane offset
    float4* dst = work + ((size_t)img << (2 * LOGN)) + (size_t)(xb * R + rp) * M * B;
    const int soff = (i * B + c) * 16 + s * (2 * M * B * 16);
#pragma unroll
    for (int m = 0; m < 16; m++)
      st4<kStream>(dst + m * T * B, soff, pair_raw(v[m]));
  }
}

template <int LAR = 0>
hipError_t launch_ifft_pre_pair14(int n_images, float4* images, float4* work, const float2* twn, const float2* twm,
                                  hipStream_t stream, int cus)
{
  constexpr int LOGN = 14;
  using S = FftShape<LOGN>;
  using P = PreCfg;
  {
    auto kern = k_cols_pre_pair14<0>;
    const int lds = P::TWM + tw_bytes<S::TW_ENTRIES>() + P::XCH;
    const int grid = persistent_grid(kern, P::WG, lds, n_images * (S::N / 2) * 2, cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(P::WG), lds, stream, n_images, images, work, twn, twm);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
      return e;
  }
  auto kern = k_rows_final<LOGN, true, LAR, kStream, 1, 0, 4, 2, 4>;
  const int lds = tw_bytes<S::TW_ENTRIES>() + lds_row_slots<LOGN>(1) * 8;
  const SlabGeom g{0, S::N};
  const int grid = persistent_grid(kern, S::T, lds, n_images * S::N, cus);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(S::T), lds, stream, n_images, g, work, images, (float*)nullptr,
                     FoamParams{}, twn);
  return hipGetLastError();
}

// The four-step EncodeIFFT (launch_ifft_fourstep) with the work slab's cache policy selectable
// (k_cols4_step1/2 WNT): ifft4bench mall.
inline hipError_t launch_ifft_fourstep_ab(int logn, int n_images, float4* images, float4* work, int wc, const float2* tw,
                                          const float2* tw2, hipStream_t stream, int cus, bool work_nt)
{
  if (logn != 14 || !tw2 || wc < 64 || (1 << logn) % wc != 0 || (wc & 63) != 0)
    return hipErrorInvalidValue;
  hipError_t e = launch_rows_ifft(logn, n_images, images, tw, stream, cus);
  if (e != hipSuccess)
    return e;
  constexpr int LOGN = 14, LOGN2 = 10, n = 1 << LOGN;
  using K2 = ColCfg<LOGN2>;
  auto k1 = work_nt ? k_cols4_step1<LOGN, true> : k_cols4_step1<LOGN, false>;
  auto k2 = work_nt ? k_cols4_step2<LOGN2, true> : k_cols4_step2<LOGN2, false>;
  const int lds2 = lds_bytes_cols<LOGN2>();
  for (int im = 0; im < n_images; im++)
    for (int x0 = 0; x0 < n; x0 += wc)
    {
      float4* img = images + ((size_t)im << (2 * LOGN));
      const int g1 = persistent_grid(k1, 256, 0, (wc / 64) * ((n / 16) / 4), cus);
      hipLaunchKernelGGL(k1, dim3(g1), dim3(256), 0, stream, 1, x0, wc, img, work, tw);
      const int g2 = persistent_grid(k2, K2::WG, lds2, 16 * (wc / K2::C), cus);
      hipLaunchKernelGGL(k2, dim3(g2), dim3(K2::WG), lds2, stream, 1, x0, wc, work, img, tw2);
      e = hipGetLastError();
      if (e != hipSuccess)
        return e;
    }
  return hipSuccess;
}


// The round-3 production k_rows_xs (the 16 CPairs formed in registers, then T_in in two halves).
template <int LOGN, int PF>
__global__ __launch_bounds__(1024) void k_rows_xs_r3(FrameParams fp, const float4* __restrict__ spec, float4* __restrict__ maps,
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
  // Source block of column u: u >> lcpr (cpr a power of two, launch_rm_rows), wave-uniform because
  // cpr is a multiple of 64: computed on the scalar unit from the wave's first column, so a load's
  // address costs one VALU mask instead of a division.
  const int lcpr = 31 - __builtin_clz(rs.cpr), cmask = rs.cpr - 1;
  const int wave0 = __builtin_amdgcn_readfirstlane((int)threadIdx.x & ~63);
  // the 8 kept elements u = m T + tid of one image: (A, B) or (D, E)
  float4 fp4[8], nx4[8];
  auto issue = [&](int item, int img, float4* p4, int m0, int m1) __attribute__((always_inline)) {
    const int c = item / rows, yl = item - c * rows;
    const size_t base = ((size_t)c * rows + yl) * rs.lp;
    const int i = opaque((int)threadIdx.x);
#pragma unroll
    for (int m = m0; m < m1; m++)
    {
      const int src = (m * T + sopaque(wave0)) >> lcpr;  // source block (scalar, computed here: not hoisted)
      const size_t sb = (size_t)src * rs.src_stride;
      p4[m] = ld4<kStream>(reinterpret_cast<const float4*>((img == 0 ? rs.ab : rs.de) + sb) + base,
                           ((m * T + i) & cmask) * 16);
    }
  };
  int item = blockIdx.x;
  if (PF > 0 && item < total)
    issue(item, 0, fp4, 0, PF);
  for (; item < total; item += gridDim.x)
  {
    const int c = item / rows, yl = item - c * rows;
    const float dk = fp.c[c].dk;
    const float sgy = (yl & 1) ? -1.0f : 1.0f;  // (-1)^q of the Nyquist-row term (rows start at an even q)
    const size_t base = ((size_t)c * rows + yl) * rs.lp;
#pragma unroll
    for (int img = 0; img < 2; img++)
    {
      const int cimg = c * 2 + img;
      const int tid = opaque((int)threadIdx.x), i = tid;
      const float4* sp = spec + (size_t)cimg * N;
      issue(item, img, fp4, PF, 8);  // the elements not prefetched
      CPair v[16];  // own lanes in v[m], the -u lanes in v[m + 8] until the transposition
#pragma unroll
      for (int m = 0; m < 8; m++)
      {
        const int u = m * T + i;
        const float kx = (float)u * dk;
        const float4 s4 = ld4<0>(sp, (N / 2 - u) * 16);  // the -u column's Nyquist-row term (x = N/2 - u)
        const int src = (m * T + sopaque(wave0)) >> lcpr;
        const float2 cc = ld2<0>(reinterpret_cast<const float2*>(rs.c + (size_t)src * rs.src_stride) + base,
                                 (u & cmask) * 8);  // C
        if (img == 0)
        {
          const CPair p = raw_pair(fp4[m]);  // (A, B)
          const float Ar = p.re.x, Ai = p.im.x, Br = p.re.y, Bi = p.im.y, Cr = cc.x, Ci = cc.y;
          v[m] = CPair{f2v{(1.0f - kx) * Ar, -Bi - kx * Cr}, f2v{(1.0f - kx) * Ai, Br - kx * Ci}};
          v[m + 8] = CPair{f2v{(1.0f + kx) * Ar + sgy * s4.x, -Bi + kx * Cr + sgy * s4.z},
                           f2v{-(1.0f + kx) * Ai + sgy * s4.y, -Br - kx * Ci + sgy * s4.w}};
        }
        else
        {
          const CPair q = raw_pair(fp4[m]);  // (D, E)
          const float Cr = cc.x, Ci = cc.y, Dr = q.re.x, Di = q.im.x, Er = q.re.y, Ei = q.im.y;
          const float kx2 = kx * kx;
          v[m] = CPair{f2v{-(Di - kx2 * Ci), -Er + kx * Di}, f2v{Dr - kx2 * Cr, -Ei - kx * Dr}};
          v[m + 8] = CPair{f2v{-(Di + kx2 * Ci) + sgy * s4.x, -Er - kx * Di + sgy * s4.z},
                           f2v{-Dr - kx2 * Cr + sgy * s4.y, Ei - kx * Dr + sgy * s4.w}};
        }
      }
      if (i == 0)
      {
        // thread 0: the Nyquist column u = -N/2 (block nyq_src, column cpr) replaces the unused -u
        // lane of u = 0 (T_in puts v[8] at n = N/2)
        const size_t ns = (size_t)rs.nyq_src * rs.src_stride;
        const float kx = -(dim / 2.0f) * dk;
        const float2 cc = ld2<kStream>(reinterpret_cast<const float2*>(rs.c + ns) + base, rs.cpr * 8);
        const float4 t = ld4<kStream>(reinterpret_cast<const float4*>((img == 0 ? rs.ab : rs.de) + ns) + base,
                                      rs.cpr * 16);
        const CPair p = raw_pair(t);
        if (img == 0)
          v[8] = CPair{f2v{(1.0f - kx) * p.re.x, -p.im.y - kx * cc.x}, f2v{(1.0f - kx) * p.im.x, p.re.y - kx * cc.y}};
        else
        {
          const float kx2 = kx * kx;
          v[8] = CPair{f2v{-(p.im.x - kx2 * cc.y), -p.re.y + kx * p.im.x}, f2v{p.re.x - kx2 * cc.x, -p.im.y - kx * p.re.x}};
        }
      }
      // the next image's fields: this row's (D, E), or the next row's (A, B) and C
      if constexpr (PF > 0)
      {
        if (img == 0)
          issue(item, 1, nx4, 0, PF);
        else if (item + (int)gridDim.x < total)
          issue(item + gridDim.x, 0, nx4, 0, PF);
      }
      // x index n = n1 + 16 n2, output k = k2 + 1024 k1: T_in gives wave n1 = w the inputs x(w + 16 n2)
      // (own lanes at n, the -u lanes at N - n, thread 0's Nyquist column at N/2); the wave's
      // 1024-point sub-transform; times W_N^(n1 k2); T_out gives thread k2 = tid the 16 values
      // Z_n1(k2); the 16-point DFT over n1 leaves v[k1] = X(tid + T k1). LDS slot of n: (n mod 16) RS + n / 16.
      const int w = tid >> 6, l = tid & 63;
      auto pslot = [&](int n) { return (n & 15) * RS + (n >> 4); };
      __syncthreads();  // the previous image's T_out reads are done
#pragma unroll
      for (int h = 0; h < 2; h++)
      {
        if (h)
          __syncthreads();
#pragma unroll
        for (int m = 0; m < 8; m++)
        {
          xs[pslot(i + m * T)] = half_of(v[m], h);
          xs[pslot(m == 0 && i == 0 ? N / 2 : N - i - m * T)] = half_of(v[m + 8], h);
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < 16; m++)
          set_half(v[m], h, xs[w * RS + l + 64 * m]);
      }
      // region w is the wave's alone until T_out's first barrier: its exchanges need no barriers
      fft_run<L2, 0, true, true>(v, l, 0, l, 0, xs + w * RS, tw2);  // v[m] = Y_w(l + 64 m)
      const float2 base_w = twiddle<LOGN>(w * l, tw);
#pragma unroll
      for (int m = 0; m < 16; m++)
        v[m] = cmul(v[m], base_w);
      apply_stage_twiddles<LOGN>(v, 64 * w, tw);  // x W_N^(w (l + 64 m))
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
      float4* dst = maps + ((size_t)cimg * rows + yl) * N;
#pragma unroll
      for (int m = 0; m < 16; m++)
        st4<kStream>(dst + m * T, tid * 16, from_pair(v[m]));
      if (img == 1)
      {
        // displacementMap (Dz, dDx/dx, dDz/dz, dDx/dz) = (re0, im0, re1, im1): Jacobian,
        // spectrum.compute:246-259
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

// Round 6: k_cols4_step2 on a resident grid (one 1024-thread workgroup per CU
// looping over items) with the vmcnt ordering of k_rows_xs EARLY: the next item's first PF loads are
// issued after this item's transform and before its 16 stores, so they do not queue behind the
// stores; the last item re-reads its own (unconditional, so the registers are not kept live across
// the loop as a second incoming value). Same arithmetic per column as production: bit-identical.
// MINB (round 6): the launch bound's second argument; 4 keeps a 512-thread (CI 8) workgroup at <= 128
// VGPRs, so two fit on a CU (without it CI 8 compiles to 134 VGPRs: one workgroup per CU).
template <int LOGN2, int PF, int CI = ColCfg<LOGN2>::C, int MINB = 1>
__global__ __launch_bounds__(FftShape<LOGN2>::T * CI, MINB) void k_cols4_step2e(int images, int x0, int wc,
                                                                         const float4* __restrict__ work,
                                                                         float4* __restrict__ img,
                                                                         const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN2>;
  constexpr int N2 = S::N, T = S::T, C = CI, LOGN = LOGN2 + 4, N = N2 * 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN2>(tw, tw_glob);
  const int c0 = threadIdx.x % C, i0 = threadIdx.x / C;
  const int strips = wc / C;
  const int total = images * 16 * strips;
  auto src_of = [&](int item) __attribute__((always_inline)) {
    const int strip = item % strips, rest = item / strips, k1 = rest & 15, im = rest >> 4;
    return work + (size_t)im * N * wc + (size_t)N2 * k1 * wc + strip * C + opaque(c0);
  };
  auto ld = [&](const float4* src, int m) __attribute__((always_inline)) {
    const f4v r = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(src + (size_t)(opaque(i0) + m * T) * wc));
    return raw_pair(make_float4(r.x, r.y, r.z, r.w));
  };
  CPair pre[PF > 0 ? PF : 1];
  if (PF > 0 && (int)blockIdx.x < total)
  {
    const float4* s0 = src_of(blockIdx.x);
#pragma unroll
    for (int m = 0; m < PF; m++)
      pre[m] = ld(s0, m);
  }
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    const int c = opaque(c0), i = opaque(i0);
    const int strip = item % strips, rest = item / strips, k1 = rest & 15, im = rest >> 4;
    const int xl = strip * C + c;
    const float4* src = src_of(item);
    CPair v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
      v[m] = m < PF ? pre[m < PF ? m : 0] : ld(src, m);
    fft_run<LOGN2, C, true>(v, i, c, xch, tw);
    if constexpr (PF > 0)
    {
      const int nx = item + (int)gridDim.x < total ? item + (int)gridDim.x : item;
      const float4* sn = src_of(nx);
#pragma unroll
      for (int m = 0; m < PF; m++)
        pre[m] = ld(sn, m);
    }
    float4* dst = img + ((size_t)im << (2 * LOGN)) + (size_t)k1 * N + x0 + xl;
#pragma unroll
    for (int m = 0; m < 16; m++)
    {
      const float4 o = from_pair(v[m]);
      __builtin_nontemporal_store(f4v{o.x, o.y, o.z, o.w}, reinterpret_cast<f4v*>(dst + (size_t)16 * (i + m * T) * N));
    }
  }
}

// Round 6: the in-place EncodeIFFT row pass (k_rows_ifft, one 1024-thread workgroup per 16384-point row)
// on a resident grid with the next row's first PF loads issued after this row's transform and before
// its 16 stores (k_rows_xs EARLY); the last row re-reads its own. Whole rows only (N = 16384, RPW 1).
template <int LOGN, int PF>
__global__ __launch_bounds__(RowCfg<LOGN>::WG, RowCfg<LOGN>::MIN_WAVES) void k_rows_ifft_early(
    int rows, float4* __restrict__ images, const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  using R = RowCfg<LOGN>;
  static_assert(R::RPW == 1, "whole rows");
  constexpr int N = S::N, T = S::T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);
  const int i0 = threadIdx.x;
  auto ld = [&](int row, int m) __attribute__((always_inline)) {
    return to_pair(ld4(images + ((size_t)row << LOGN) + ((m + 8) & 15) * T, opaque(i0) * 16));
  };
  CPair pre[PF > 0 ? PF : 1];
  if (PF > 0 && (int)blockIdx.x < rows)
  {
#pragma unroll
    for (int m = 0; m < PF; m++)
      pre[m] = ld(blockIdx.x, m);
  }
  for (int row = blockIdx.x; row < rows; row += gridDim.x)
  {
    const int i = opaque(i0);
    CPair v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
      v[m] = m < PF ? pre[m < PF ? m : 0] : ld(row, m);
    fft_run<LOGN, 0, R::SPLIT>(v, i, 0, xch, tw);
    if constexpr (PF > 0)
    {
      const int nx = row + (int)gridDim.x < rows ? row + (int)gridDim.x : row;
#pragma unroll
      for (int m = 0; m < PF; m++)
        pre[m] = ld(nx, m);
    }
    float4* line = images + ((size_t)row << LOGN);
#pragma unroll
    for (int m = 0; m < 16; m++)
      st4(line + m * T, i * 16, from_pair(v[m]));
  }
}

// Round 6: the 16384 four-step work slab blocked in strips of 16 columns, [strip][N rows][16], so that
// step 2's item (k1, strip) reads one contiguous 256-KiB run (1 KiB per wave load) instead of 256-B
// pieces 32 KiB apart; step 1 then stores 256-B pieces (4 per wave store) instead of 1-KiB runs.
// Same arithmetic as k_cols4_step1 / k_cols4_step2: bit-identical images.
template <int LOGN>
__global__ __launch_bounds__(256) void k_cols4_step1b(int images, int x0, int wc, const float4* __restrict__ img,
                                                      float4* __restrict__ work, const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  constexpr int N = S::N, N2 = N / 16;
  __shared__ float2 tw[S::TW_ENTRIES];
  load_twiddles<LOGN>(tw, tw_glob);
  const int xblocks = wc / 64;
  const int total = images * xblocks * (N2 / 4);
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int t = item;
    const int xbk = t % xblocks;
    t /= xblocks;
    const int n2 = (t % (N2 / 4)) * 4 + wv, im = t / (N2 / 4);
    const int xl = xbk * 64 + lane;
    const float4* src = img + ((size_t)im << (2 * LOGN)) + x0 + xl;
    CPair v[16];
#pragma unroll
    for (int n1 = 0; n1 < 16; n1++)
    {
      const f4v r = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(src + (size_t)(N2 * ((n1 + 8) & 15) + n2) * N));
      v[n1] = to_pair(make_float4(r.x, r.y, r.z, r.w));
    }
    idft16(v);
    apply_stage_twiddles<LOGN>(v, n2, tw);
    float4* dst = work + (size_t)im * N * wc + (size_t)(xl >> 4) * N * 16 + (xl & 15);
#pragma unroll
    for (int k1 = 0; k1 < 16; k1++)
    {
      const float4 o = pair_raw(v[k1]);
      __builtin_nontemporal_store(f4v{o.x, o.y, o.z, o.w}, reinterpret_cast<f4v*>(dst + (size_t)(N2 * k1 + n2) * 16));
    }
  }
}

template <int LOGN2, int CI = ColCfg<LOGN2>::C>
__global__ __launch_bounds__(FftShape<LOGN2>::T * CI) void k_cols4_step2b(int images, int x0, int wc,
                                                                         const float4* __restrict__ work,
                                                                         float4* __restrict__ img,
                                                                         const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN2>;
  constexpr int N2 = S::N, T = S::T, C = CI, LOGN = LOGN2 + 4, N = N2 * 16;
  static_assert(C == 16, "16-column strips");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN2>(tw, tw_glob);
  const int c0 = threadIdx.x % C, i0 = threadIdx.x / C;
  const int strips = wc / C;
  const int total = images * 16 * strips;
  auto src_of = [&](int item) __attribute__((always_inline)) {
    const int strip = item % strips, rest = item / strips, k1 = rest & 15, im = rest >> 4;
    return work + (size_t)im * N * wc + ((size_t)strip * N + (size_t)N2 * k1) * 16 + opaque(c0);
  };
  auto ld = [&](const float4* src, int m) __attribute__((always_inline)) {
    const f4v r = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(src + (size_t)(opaque(i0) + m * T) * 16));
    return raw_pair(make_float4(r.x, r.y, r.z, r.w));
  };
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    const int c = opaque(c0), i = opaque(i0);
    const int strip = item % strips, rest = item / strips, k1 = rest & 15, im = rest >> 4;
    const int xl = strip * C + c;
    const float4* src = src_of(item);
    CPair v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
      v[m] = ld(src, m);
    fft_run<LOGN2, C, true>(v, i, c, xch, tw);
    float4* dst = img + ((size_t)im << (2 * LOGN)) + (size_t)k1 * N + x0 + xl;
#pragma unroll
    for (int m = 0; m < 16; m++)
    {
      const float4 o = from_pair(v[m]);
      __builtin_nontemporal_store(f4v{o.x, o.y, o.z, o.w},
                                  reinterpret_cast<f4v*>(dst + (size_t)16 * (i + m * T) * N));
    }
  }
}

}  // namespace oceanfft
