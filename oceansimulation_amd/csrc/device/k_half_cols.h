// device/k_half_cols.h — the half-spectrum column pass (whole grids of 1024 .. 4096, and the
// strip-dealt slabs): evolve (resources/spectrum.compute:183-240) + the y iFFT of the five Hermitian
// field multiples of H.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ocean_internal.h"
#include "device/evolve.h"
#include "device/fft.h"
#include "device/grid.h"
#include "device/lane_xchg.h"
#include "device/memory.h"
#include "device/spectrum.h"

namespace oceanfft
{

// ------------------------------------------------------------------------------------------------
// Generator path, half spectrum (whole grids, B = 4, one strip per pass-1 item: N = 1024 .. 4096).
// All eight output fields are real multipliers of the one Hermitian field H (tests/
// half_spectrum_ref.py): lane0 = (1 - kx) A, lane1 = i B - kx C, lane2 = i (D - kx^2 C),
// lane3 = -E - i kx D with A = H, B = kz H, C = H/|k|, D = kz H/|k|, E = kz^2 H/|k|. The kx factors
// commute with the y transform, and H(-k) = conj(H(k)) makes each y-transformed field
// (anti-)Hermitian in u = x - N/2, so pass 1 transforms only the columns u >= 0 and the Nyquist
// column u = -N/2 (half the columns, half of h0 read), storing 5 complex fields (20 B per grid
// point instead of 32); pass 2 rebuilds u < 0 as s_F conj(G_F(q, -u)). The reference's Nyquist row
// is not Hermitian-paired (its partner is evaluated at +N/2, spectrum.compute:165); its share is the
// rank-1 term (-1)^q R(p), R the x-transform of a one-row spectrum built by k_half_nyquist.
// Frame bytes: h0 8 + fields 20 + 20 + maps 32 + Jacobian 4 = 84 per point (the full path: 116).
// ------------------------------------------------------------------------------------------------

template <int LOGN>
struct HalfCfg
{
  static constexpr int N = 1 << LOGN;
  static constexpr int B = ColFirstCfg<LOGN>::B;
  static constexpr int STRIPS = N / (2 * B) + 1;  // u in [0, N/2), then the strip of x = 0..B-1
  static constexpr bool SUPPORTED = B == 4 && ColFirstCfg<LOGN>::SPW == 1;  // blocked whole-grid path
  static constexpr bool SLAB_SUPPORTED = ColFirstCfg<LOGN>::SPW == 1;      // strip-dealt path, any B
};

// Whole-grid half-spectrum field layout, texel offset of (row y, strip, column b of the strip) in a
// cascade. RG = 1: strips [strip][y][B], a strip one contiguous run (pass 1 stores 1-KiB wave runs,
// pass 2 reads one RPW * B-texel piece per strip). RG > 1: row groups [y / RG][strip][y % RG][B], so a
// pass-2 item of RG rows reads one contiguous run and pass 1 stores RG * B-texel pieces. The offset is
// linear in (y, strip) for y a multiple of RG: offset(y0 + i, s, b) = offset(y0, s) + offset(i, 0, b).
// Production: RG = 2, RGC = 4. A pass-2 item (2 rows) reads whole 128-B lines of gab/gde in one
// contiguous run per image, and gc's 128-B lines are shared by the two items paired on one XCD
// (xcd_pair_slot); pass 1 stores 128-B pieces. Against strips (RG = 1): pass 2 1.637 -> 1.506 ms,
// pass 1 0.934 -> 0.960 ms, frame 2.581 -> 2.477 ms at 8 x 4096^2 (tools/microbench/halfbench).
constexpr int kHalfRG = 2, kHalfRGC = 4;
// Pass 1's H pairs outside the scratch (k_cols_half HL / HK): one pair per thread in the LDS the
// exchange leaves free, four in VGPRs (128 VGPRs at N = 4096, no spills); the scratch keeps 3 of 8.
// 0.945 -> 0.817 ms per 8 x 4096^2, frame 2.332 -> 2.206 ms, fields bit-identical (halfbench hkeep).
constexpr int kHalfHL = 1, kHalfHK = 4, kHalfHKSeed = 2;  // the fused re-seed frame: variant 33 = all in scratch
// FB: columns per field strip (4 = the h0 strip; 2 = k_cols_half2's half strips, FS = 2 STRIPS).
template <int LOGN, int RG, int FB = 4>
__device__ __forceinline__ int half_group_offset(int y, int strip, int b = 0)
{
  constexpr int N = HalfCfg<LOGN>::N, FS = HalfCfg<LOGN>::STRIPS * HalfCfg<LOGN>::B / FB;
  return RG == 1 ? (strip * N + y) * FB + b : (((y / RG) * FS + strip) * RG + (y % RG)) * FB + b;
}

// HX: the y transform of a 4096-point column (B = 4 columns per 1024-thread workgroup) with one LDS
// exchange instead of fft_run's two. Thread t = 64 w + 4 a + b holds x(n) of column b at n = a + 16 w +
// 256 m in v[m] (the production load order); with k = k0 + 16 k1 + 256 k2,
//   W^(nk) = W_16^(m k0) . W_N^((a + 16 w) k0) . W_16^(w k1) . W_256^(a k1) . W_16^(a k2):
// a DFT-16 over m in registers, twiddle, an LDS transposition of (register k0, wave w) — slot
// (k0 16 + w) 64 + lane, 64 consecutive 8-B slots per access, conflict-free — a DFT-16 over w, twiddle,
// the in-wave transposition register bits 0..3 <-> lane bits 2..5 (lane_xchg.h: v_permlane16/32_swap +
// DPP) and a DFT-16 over a. On exit v[m] = X(w + 16 a + 256 m): rows i2 + m T with i2 = w + 16 a. Two
// split halves of 128 KiB, 4 barriers per round against fft_run's 8.
// HX 2's storage row of row y (and its inverse): y = k0 + 16 k1 + 256 k2 -> 256 k0 + 16 k2 + k1.
__host__ __device__ constexpr int hx_store_row(int y) { return ((y & 15) << 8) | ((y >> 8) << 4) | ((y >> 4) & 15); }
__host__ __device__ constexpr int hx_row_of_store(int s) { return (s >> 8) | ((s & 15) << 4) | (((s >> 4) & 15) << 8); }

__device__ __forceinline__ void fft_cols_hx(CPair* v, int t, void* lds, const float2* __restrict__ tw)
{
  constexpr int LOGN = 12;
  float2* xs = reinterpret_cast<float2*>(lds);
  const int w = t >> 6, lane = t & 63, a = (t >> 2) & 15;
  idft16(v);
  apply_stage_twiddles<LOGN>(v, a + 16 * w, tw);  // x W_N^((a + 16 w) k0)
#pragma unroll
  for (int h = 0; h < 2; h++)
  {
    __syncthreads();  // the previous reads of the region are done
#pragma unroll
    for (int k0 = 0; k0 < 16; k0++)
      xs[(k0 * 16 + w) * 64 + lane] = half_of(v[k0], h);
    __syncthreads();
#pragma unroll
    for (int ww = 0; ww < 16; ww++)  // this wave is now k0 = w
      set_half(v[ww], h, xs[(w * 16 + ww) * 64 + lane]);
  }
  idft16(v);                                      // v[k1]
  apply_stage_twiddles<LOGN>(v, 16 * a, tw);      // x W_256^(a k1)
  transpose_reg_lanes_2_5(v);                     // v[a'], lane bits 2..5 = k1
  idft16(v);                                      // v[k2] = X(w + 16 a + 256 k2)
}

// Pass 1: per strip of B columns (u >= 0, or the Nyquist strip), three y-iFFT rounds of CPairs:
// (A, B), (D, E), (C, 0), stored as gab, gde (float4) and gc (float2): pass 2 reads (A, B) + C for
// image 0 and C + (D, E) for image 1. H is re-evolved per round from h0: keeping the 16 H (32 VGPRs)
// next to the transform's ~107 spills in a 1024-thread workgroup.
// HS (H scratch): round 0 evolves H once and parks it in a per-workgroup scratch slice (8 B per
// texel, [m][thread], L2/MALL-resident); rounds 1 and 2 load it back (nt: served by L2, never a
// stale L1 line from the previous item) instead of re-reading h0 (16 B) and re-evolving.
// SLAB (strip-dealt layout, HalfSlab): this rank transforms global strips [strip0, strip0 +
// nstrips) and writes its output in destination-block order into `send` (block q = rows
// [q w, q w + w): gab | gde | gc parts of C * S * w * B elements, element ((c S + sl) w + yl) B + b),
// so one equal-split all-to-all hands every rank the rows of its row pass. h0 is the whole grid's
// blocked image when h0_full, else the rank's strips in order ([c][sl][N][B]).
// SEED (the fused re-seed frame, CalculateOcean(dt, true) on whole grids): round 0 evaluates each
// texel's two amplitudes (seed[c], the host's settings constants) instead of loading h0, so h0 is
// neither written nor read this frame (HS only).
// RG / RGC (whole grids): rows per group of the gab/gde and the gc layout (half_group_offset).
// CPI: columns per item (B = the whole strip; B / 2: half strips, T * CPI threads, two workgroups
// per CU so one's loads and stores overlap the other's transform; the strip's two halves are items
// 2p, 2p + 1 on one XCD, whose loads share h0 lines). Production at <= 2 cascades with FB = 2
// (half_fields_fb); on the 4-column layout the halves' stores are half lines (slower).
// HP: the H scratch holds pairs (H(m), H(m + 1)) per thread in 16-B entries ([m / 2][thread]): 8
// stores and 16 loads of 16 B per item instead of 16 and 32 of 8 B.
// PC (packed C round, needs HS + HP and whole strips of B >= 2): round 2's CPair (C, 0) wastes its
// second lane, so the first half of the workgroup transforms the strip's column pairs (2 p, 2 p + 1)
// as (C_2p, C_2p+1) instead (CI = B / 2 interleaved transforms, H of both columns from the scratch
// entries round 0 wrote) and stores 16-B gc pairs; the second half only matches the transform's
// barriers. Per lane the arithmetic is the unpacked round's, so the fields are bit-identical.
// HL / HK (HP only): of the thread's 8 H pairs, pairs [0, HL) live in the LDS left over by the exchange
// (16 B per thread each, after K::LDS1) and pairs [HL, HL + HK) in VGPRs from round 0 to round 2; only
// the rest goes through the scratch. The scratch's HBM traffic (its lines are written back and, about
// half of them, re-fetched: 1.30x algorithmic) costs 0.118 of 0.912 ms (halfbench_nohs).
// HX (N = 4096, whole strips): the transform is fft_cols_hx; 1: the thread stores rows i2 + m T; 2
// (whole grids, RG > 1): the fields hold row y = k0 + 16 k1 + 256 k2 at storage row hx_store_row(y) =
// 256 k0 + 16 k2 + k1, so each store instruction writes 16 consecutive storage rows (whole lines);
// the row pass reads storage rows (k_rows_hp YP).
// FB (half strips, whole grids): the fields are FB = CPI columns wide (half_group_offset<.., FB>), so a
// half-strip item's stores are whole lines when RG * FB * 16 B = 128 B (gab, gde) and RGC * FB * 8 B
// = 128 B (gc); the row pass reads the same layout (k_rows_hp FB).
// PUT (SLAB only; the one-sided exchange, ocean_peers): `send` is then the device table of the ranks'
// destinations, ((const uint64_t*)send)[q] = this rank's block in rank q's receive slot, and block q
// is stored there instead of at send + q * block bytes.
// EARLY (round 5; a wave retires its memory instructions in issue order, so a load issued after the
// round's field stores waits for them): bit 0, the scratch pairs of round r + 1 are loaded before
// round r's stores (HS + HP); bits 1 / 2, the first 8 / all 16 h0 texels of the workgroup's next item
// before round 2's stores (whole strips; the first item's in a prologue).
// QX (round 6): the transform's LDS exchanges move one float at a time (fft.h QUARTER: 68 KiB instead of
// 136 KiB at 4096, twice the barriers), so up to 5 of the thread's 8 H pairs fit in the LDS (HL) beside
// HK in VGPRs: with HL + HK = 8 nothing goes through the scratch, and rounds 1 and 2 start on LDS reads
// instead of scratch loads that a wave's vmcnt orders behind the previous round's field stores.
// DELAY: see the kernel body (an A/B probe; production 0).
// RSPLIT (round 6, small grids): one work slot per (item, field round), so the three rounds of a strip
// run on three workgroups at once (each re-reads h0 and re-evolves H: 16 B of h0 per kept texel and
// round instead of once); the slots of a strip sit on one XCD (xcd_group_slot<3>) so the two repeat
// reads of its h0 lines are L2 hits. For grids whose column pass is one item's latency long (2048^2
// with one cascade: 257 items on 512 workgroup slots).
// NYQ (whole grids): the Nyquist-row term (k_half_nyquist's spec, written to `send` as float4[C][2][N])
// is computed by the workgroup of the last item slot, which has the fewest items, after them: one
// launch per frame fewer (half_nyquist_texel, the same arithmetic as the kernel the slab paths use).
// HB (half strips, whole grids): h0's strip width. HB = CPI = 2: h0 is blocked in 2-column strips, so a
// half-strip item reads its own contiguous strip instead of the 32-B halves of 64-B row pieces that
// its partner item reads the other halves of (launch_half_columns at <= 2 cascades: 0.122 -> 0.114 ms
// per 4096^2 cascade, 0.935 -> 0.792 ms per 8, halfbench fb2h).
template <int LOGN, int LA = 0, int SA = kStream, bool HS = false, bool SLAB = false, bool SEED = false, int RG = 1,
          int RGC = 1, int CPI = ColFirstCfg<LOGN>::B, bool HP = false, bool PC = false, int HL = 0, int HK = 0,
          int HX = 0, int FB = 4, bool PUT = false, int HB = ColFirstCfg<LOGN>::B, int EARLY = 0, bool NYQ = false,
          bool QX = false, int DELAY = 0, bool RSPLIT = false>
__global__ __launch_bounds__(FftShape<LOGN>::T * CPI, CPI < ColFirstCfg<LOGN>::B ? 4 : 1) void k_cols_half(FrameParams fp, const float4* __restrict__ h0,
                                                                     float4* __restrict__ gab, float4* __restrict__ gde,
                                                                     float2* __restrict__ gc,
                                                                     const float2* __restrict__ tw_glob,
                                                                     float2* __restrict__ hs, HalfSlab hsl,
                                                                     unsigned char* __restrict__ send, int h0_full,
                                                                     const SpectrumConsts* __restrict__ seed)
{
  using S = FftShape<LOGN>;
  using K = ColFirstCfg<LOGN>;
  using HC = HalfCfg<LOGN>;
  constexpr int N = S::N, T = S::T, B = K::B, STRIPS = HC::STRIPS, WG = T * CPI, HALVES = B / CPI;
  static_assert(SLAB ? HC::SLAB_SUPPORTED : HC::SUPPORTED, "half-spectrum path: one strip per item (B = 4 unless SLAB)");
  static_assert(CPI * HALVES == B && HALVES <= 2 && (HALVES == 1 || !SLAB), "whole or half strips");
  static_assert((HL == 0 && HK == 0) || (HS && HP && !PC && HL + HK <= 8), "H pairs outside the scratch");
  static_assert(!HX || (LOGN == 12 && CPI == 4 && B == 4 && !PC), "HX: 4096-point columns, whole 4-column strips");
  static_assert(HX != 2 || (!SLAB && RG > 1 && RGC > 1), "HX 2: whole-grid row-group layouts");
  constexpr int MSTEP = HX == 2 ? 16 : T;  // storage rows between v[m] and v[m + 1]
  static_assert(FB == 4 || (FB == CPI && HALVES == 2 && !SLAB && RG > 1 && RGC > 1 && !HX), "FB: half-strip fields");
  static_assert(!PUT || (SLAB && !PC), "PUT: the strip-dealt slab stores");
  static_assert(HB == B || (HB == CPI && HALVES == 2 && !SLAB), "HB: half strips over 2-column h0 strips");
  static_assert(!NYQ || !SLAB, "NYQ: whole grids (send is the spec output)");
  static_assert(!QX || (!HX && !PC), "QX: the fft_run transform");
  constexpr int XB = CPI * S::PADDED * (QX ? 4 : 8);  // the exchange's bytes (K::LDS1 for whole strips; half with QX)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  float4* hlds = reinterpret_cast<float4*>(static_cast<unsigned char*>(xch) + XB);  // HL pairs [p][thread]
  load_twiddles<LOGN>(tw, tw_glob);
  if constexpr (DELAY > 0)
    if ((int)blockIdx.x >= (int)gridDim.x / 2)
    {
      // DELAY (round 6, tools/microbench A/B): the second half of a two-per-CU grid starts DELAY
      // wall-clock ticks (100 MHz) late, so the two workgroups of a CU run their store phases out of step
      const long long t0 = wall_clock64();
      while (wall_clock64() - t0 < DELAY)
        __builtin_amdgcn_s_sleep(8);
    }

  const int nstrips = SLAB ? hsl.nstrips : STRIPS;
  const int total = fp.cascades * nstrips * HALVES;
  static_assert(!RSPLIT || (!HS && !SEED && !SLAB && HALVES == 1 && EARLY == 0 && !PC && !HX),
                "RSPLIT: whole strips, h0 re-read per round");
  constexpr int RS3 = RSPLIT ? 3 : 1;  // work slots per item
  const float dim = (float)N;
  constexpr int NPRE = 8 - HL - HK;  // scratch pairs per round (HP)
  constexpr bool EPAIR = (EARLY & 1) && HS && HP && !PC && NPRE > 0;
  constexpr int EH0 = (EARLY & 4) ? 16 : (EARLY & 2) ? 8 : 0;
  static_assert(EH0 == 0 || (HALVES == 1 && HS && !SEED && !PC), "EARLY h0: whole strips");
  float4 hpre[EPAIR ? NPRE : 1];  // EARLY 1: the next round's scratch pairs
  float4 apre[EH0 > 0 ? EH0 : 1];  // EARLY 2 / 4: the next item's first h0 texels
  // h0 of item `it` (whole strips): the strip's base and this thread's offset in it
  auto h0_of = [&](int it, const float4*& sp, int& lo) __attribute__((always_inline)) {
    const int c2 = it / nstrips, s2 = it - c2 * nstrips;
    const int sg2 = SLAB ? hsl.strip0 + s2 : s2;
    const int xb2 = sg2 == STRIPS - 1 ? 0 : N / (2 * B) + sg2;
    sp = (!SLAB || h0_full) ? h0 + ((size_t)c2 * (N / B) + xb2) * N * B : h0 + ((size_t)c2 * nstrips + s2) * N * B;
    const int t2 = opaque((int)threadIdx.x);
    lo = (((t2 / CPI) % T) * B + t2 % CPI) * 16;
  };
  if constexpr (EH0 > 0)
    if ((int)blockIdx.x < total)
    {
      const float4* sp;
      int lo;
      h0_of(blockIdx.x, sp, lo);
#pragma unroll
      for (int m = 0; m < EH0; m++)
        apre[m] = ld4s<LA>(sp, lo, ((m + 8) & 15) * T * B * 16);
    }
  for (int slot = RSPLIT ? xcd_group_slot<3>(blockIdx.x, gridDim.x) : HALVES > 1 ? xcd_pair_slot(blockIdx.x, gridDim.x)
                                                                              : (int)blockIdx.x;
       slot < total * RS3; slot += gridDim.x)
  {
    const int item = RSPLIT ? slot / 3 : slot;
    const int hh = HALVES > 1 ? item % HALVES : 0, si = HALVES > 1 ? item / HALVES : item;
    const int c = si / nstrips, s = si - c * nstrips;  // s: the rank's strip index
    const int sg = SLAB ? hsl.strip0 + s : s;           // global strip
    if (HALVES > 1 && sg == STRIPS - 1 && hh != 0)
      continue;  // Nyquist strip: only column 0 (u = -N/2) is kept (uniform per workgroup)
    const int b = opaque((int)threadIdx.x) % CPI + hh * CPI;  // column within the strip
    const int xb = sg == STRIPS - 1 ? 0 : N / (2 * B) + sg;
    const CascadeFrame f = fp.c[c];
    const float4* src = HB != B                  ? h0 + ((size_t)c * (N / HB) + xb * (B / HB) + hh) * N * HB
                        : (!SLAB || h0_full) ? h0 + ((size_t)c * (N / B) + xb) * N * B
                                             : h0 + ((size_t)c * nstrips + s) * N * B;
    // the strip's first texel in the cascade's fields (whole grids); + half_group_offset(m T, 0) per m
    const int fs = FB == 4 ? s : 2 * s + hh;  // field strip
    const size_t gbase = RG == 1 ? ((size_t)c * STRIPS + s) * N * B
                                 : (size_t)c * STRIPS * N * B + half_group_offset<LOGN, RG, FB>(0, fs);
    const size_t cgbase = RGC == 1 ? ((size_t)c * STRIPS + s) * N * B
                                   : (size_t)c * STRIPS * N * B + half_group_offset<LOGN, RGC, FB>(0, fs);
    const int bf = FB == 4 ? b : b - hh * CPI;  // column within the field strip
    const int x = xb * B + b;
    float4 hk[HK > 0 ? HK : 1];  // HK: H pairs kept in VGPRs across the rounds
    // one field round: (A, B), (D, E) or (C, 0) of the 16 texels, y-iFFT, store
    auto run_round = [&](int round) __attribute__((always_inline)) {
      const int i = (opaque((int)threadIdx.x) / CPI) % T;
      const int voff = (i * B + b) * 16;
      CPair v[16];
      auto pack = [&](int m, float2 H, const KVec& q) __attribute__((always_inline)) {
        if (round == 0)  // (A, B) = (H, kz H)
          v[m] = CPair{f2v{H.x, q.kz * H.x}, f2v{H.y, q.kz * H.y}};
        else if (round == 1)  // (D, E) = (kz H / |k|, kz^2 H / |k|)
        {
          const float e = q.kz * q.dirz;
          v[m] = CPair{f2v{q.dirz * H.x, e * H.x}, f2v{q.dirz * H.y, e * H.y}};
        }
        else  // (C, 0) = (H / |k|, 0)
          v[m] = CPair{f2v{q.inv * H.x, 0.0f}, f2v{q.inv * H.y, 0.0f}};
      };
      if (SEED && round == 0)
      {
        static_assert(!SEED || HS, "the fused seed keeps H in the scratch");
        float2* hsb = hs + (size_t)blockIdx.x * 16 * WG;
        const int hoff = opaque((int)threadIdx.x) * 8;
        const SpectrumConsts q = seed[c];
        // the evaluator is too large to unroll 16 times: a rolled loop parks each H in the scratch,
        // then the round reads them back like rounds 1 and 2 (its own stores, from L2)
#pragma unroll 1
        for (int m = 0; m < 16; m++)
        {
          const int y = i + ((m + 8) & 15) * T;
          const float2 H = evolve(seed_texel(q, x, y, dim), make_kvec(x, y, dim, f.dk).k, f);
          if (HP && (m >> 1) < HL)  // HL pairs: the LDS slot (a dynamic index is fine there)
            reinterpret_cast<float2*>(hlds)[((m >> 1) * WG + threadIdx.x) * 2 + (m & 1)] = H;
          else if constexpr (HP)
            st2s<0>(hsb, hoff * 2 + (m & 1) * 8, (m >> 1) * WG * 16, H);
          else
            st2s<0>(hsb, hoff, m * WG * 8, H);
        }
        __threadfence_block();  // this thread's scratch stores are complete before it reads them back
        if constexpr (HP)
        {
          // read back by pairs; the HK pairs stay in VGPRs for rounds 1 and 2
#pragma unroll
          for (int m = 0; m < 16; m += 2)
          {
            const int y = i + ((m + 8) & 15) * T, p = m >> 1;
            const float4 pp = p < HL ? hlds[p * WG + threadIdx.x] : ld4s<kStream>(hsb, hoff * 2, p * WG * 16);
            if (p >= HL && p < HL + HK)
              hk[p < HL + HK && p >= HL ? p - HL : 0] = pp;
            pack(m, make_float2(pp.x, pp.y), make_kvec(x, y, dim, f.dk));
            pack(m + 1, make_float2(pp.z, pp.w), make_kvec(x, y + T, dim, f.dk));
          }
        }
        else
        {
#pragma unroll
          for (int m = 0; m < 16; m++)
          {
            const int y = i + ((m + 8) & 15) * T;
            pack(m, ld2s<kStream>(hsb, hoff, m * WG * 8), make_kvec(x, y, dim, f.dk));
          }
        }
      }
      else if (!HS || round == 0)
      {
        float2* hsb = hs + (size_t)blockIdx.x * 16 * WG;
        const int hoff = opaque((int)threadIdx.x) * 8;
        float4 a[16];
        float2 hprev = make_float2(0.0f, 0.0f);
#ifdef OCEAN_ABLATE_H0LOAD  // timing ablation (tools/microbench): every item reads cascade 0's strip 0 (L2-resident)
        const float4* srcl = h0;
#else
        const float4* srcl = src;
#endif
        // HB = 2: the half strip's own 2-column h0 strip (contiguous 32-B row pieces)
        const int loff = HB == B ? voff : (i * HB + (b - hh * CPI)) * 16;
#pragma unroll
        for (int m = 0; m < 16; m++)  // fftShift on y folded into the load
          a[m] = m < EH0 ? apre[m < EH0 ? m : 0] : ld4s<LA>(srcl, loff, ((m + 8) & 15) * T * HB * 16);
#pragma unroll
        for (int m = 0; m < 16; m++)
        {
          const int y = i + ((m + 8) & 15) * T;
          const KVec q = make_kvec(x, y, dim, f.dk);
          const float2 H = evolve(a[m], q.k, f);
#ifndef OCEAN_ABLATE_HS
          if (HS && HP)
          {
            const int p = m >> 1;
            if ((m & 1) && p < HL)
              hlds[p * WG + threadIdx.x] = make_float4(hprev.x, hprev.y, H.x, H.y);
            else if ((m & 1) && p < HL + HK)
              hk[p - HL] = make_float4(hprev.x, hprev.y, H.x, H.y);
            else if (m & 1)
              st4s<0>(hsb, hoff * 2, p * WG * 16, make_float4(hprev.x, hprev.y, H.x, H.y));
            else
              hprev = H;
          }
          else if (HS)
            st2s<0>(hsb, hoff, m * WG * 8, H);
#else
          (void)hsb;
          (void)hoff;
#endif
          pack(m, H, q);
        }
      }
      else
      {
        const float2* hsb = hs + (size_t)blockIdx.x * 16 * WG;
        const int hoff = opaque((int)threadIdx.x) * 8;
#pragma unroll
        for (int m = 0; m < 16; m++)
        {
          const int y = i + ((m + 8) & 15) * T;
#ifdef OCEAN_ABLATE_HS  // timing ablation (tools/microbench): no scratch read-back, wrong results
          (void)hsb;
          pack(m, make_float2((float)hoff, (float)m), make_kvec(x, y, dim, f.dk));
#else
          if constexpr (HP)
          {
            if ((m & 1) == 0)
            {
              const int pi = m >> 1;
              const float4 p = pi < HL        ? hlds[pi * WG + threadIdx.x]
                               : pi < HL + HK ? hk[pi < HL + HK ? pi - HL : 0]
                               : EPAIR        ? hpre[pi >= HL + HK ? pi - HL - HK : 0]
                                              : ld4s<kStream>(hsb, hoff * 2, pi * WG * 16);
              pack(m, make_float2(p.x, p.y), make_kvec(x, y, dim, f.dk));
              pack(m + 1, make_float2(p.z, p.w), make_kvec(x, y + T, dim, f.dk));
            }
          }
          else
            pack(m, ld2s<kStream>(hsb, hoff, m * WG * 8), make_kvec(x, y, dim, f.dk));
#endif
        }
      }
      int io = i;  // the thread's output rows io + m T
      if constexpr (HX)
      {
        const int t = opaque((int)threadIdx.x);
        fft_cols_hx(v, t, xch, tw);
        io = HX == 2 ? 256 * (t >> 6) + ((t >> 2) & 15) : (t >> 6) + 16 * ((t >> 2) & 15);
      }
      else
      {
        const int reg = HALVES > 1 ? opaque((int)threadIdx.x) % CPI : b;
        fft_run<LOGN, CPI, true, false, QX>(v, i, reg, i, reg, xch, tw);
      }
      if constexpr (EPAIR)
        if (round < 2)  // the next round's scratch pairs, before this round's stores
        {
          const float2* hsb = hs + (size_t)blockIdx.x * 16 * WG;
          const int hoff = opaque((int)threadIdx.x) * 8;
#pragma unroll
          for (int p = 0; p < NPRE; p++)
            hpre[p] = ld4s<kStream>(hsb, hoff * 2, (HL + HK + p) * WG * 16);
        }
      if constexpr (EH0 > 0)
        if (round == 2)  // the next item's first h0 texels, before this round's stores (unconditional:
        {                // the last item re-reads its own, so the consumed registers are not kept live)
          const float4* sp;
          int lo;
          h0_of(item + (int)gridDim.x < total ? item + (int)gridDim.x : item, sp, lo);
#pragma unroll
          for (int m = 0; m < EH0; m++)
            apre[m] = ld4s<LA>(sp, lo, ((m + 8) & 15) * T * B * 16);
        }
      const int vo = (io * B + b) * 16;
#pragma unroll
      for (int m = 0; m < 16; m++)
      {
#ifdef OCEAN_ABLATE_FSTORE  // timing ablation (tools/microbench): the field stores skipped, values kept live
        asm volatile("" ::"v"(v[m].re), "v"(v[m].im));
        if (m >= 0)
          continue;
#endif
        if constexpr (SLAB)
        {
          // row y = m T + io lies in block q = m T / w (w is a multiple of T), at yl = m T % w + io
          const size_t part = (size_t)fp.cascades * hsl.S * hsl.w * B;  // elements per part
          const int q = (m * T) / hsl.w, yl0 = (m * T) % hsl.w;
          const size_t el = (((size_t)c * hsl.S + s) * hsl.w + yl0) * B;
          // block = the three parts, then the Nyquist-row term [c][2][N] (half_slab_block_bytes).
          // The block base is built at its store (sopaque): hoisted, the 16 descriptors spilled SGPRs.
          unsigned char* blk =
              PUT ? reinterpret_cast<unsigned char*>(sopaque((size_t)reinterpret_cast<const uint64_t*>(send)[q]))
                  : send + sopaque((size_t)q * (part * 40 + (size_t)fp.cascades * 2 * N * 16));
          if (round == 0)
            st4<SA>(blk + el * 16, vo, pair_raw(v[m]));
          else if (round == 1)
            st4<SA>(blk + part * 16 + el * 16, vo, pair_raw(v[m]));
          else
            st2<SA>(blk + part * 32 + el * 8, (io * B + b) * 8, make_float2(v[m].re.x, v[m].im.x));
        }
        else if constexpr (RG == 1 && RGC == 1)
        {
          if (round == 0)
            st4s<SA>(gab + gbase, vo, m * T * B * 16, pair_raw(v[m]));
          else if (round == 1)
            st4s<SA>(gde + gbase, vo, m * T * B * 16, pair_raw(v[m]));
          else
            st2s<SA>(gc + gbase, (io * B + b) * 8, m * T * B * 8, make_float2(v[m].re.x, v[m].im.x));
        }
        else if (round == 0)  // one descriptor per field; the row group of m T in soffset
          st4s<SA>(gab + gbase, half_group_offset<LOGN, RG, FB>(io, 0, bf) * 16, half_group_offset<LOGN, RG, FB>(m * MSTEP, 0) * 16,
                   pair_raw(v[m]));
        else if (round == 1)
          st4s<SA>(gde + gbase, half_group_offset<LOGN, RG, FB>(io, 0, bf) * 16, half_group_offset<LOGN, RG, FB>(m * MSTEP, 0) * 16,
                   pair_raw(v[m]));
        else
          st2s<SA>(gc + cgbase, half_group_offset<LOGN, RGC, FB>(io, 0, bf) * 8, half_group_offset<LOGN, RGC, FB>(m * MSTEP, 0) * 8,
                   make_float2(v[m].re.x, v[m].im.x));
      }
    };
    // PC: round 2 as (C_2p, C_2p+1) pairs on the first half of the workgroup (see the template note)
    auto run_round_c = [&]() __attribute__((always_inline)) {
      constexpr int BP = B > 1 ? B / 2 : 1, NBAR = (S::NSTAGE - 1) * 4;  // split exchanges: 2 halves x 2 barriers
      static_assert(!PC || (HS && HP && HALVES == 1 && B >= 2 && (WG / 2) % 64 == 0), "packed C round");
      if (__builtin_amdgcn_readfirstlane((int)threadIdx.x) >= WG / 2)  // wave-uniform (scalar) branch
      {
#pragma unroll 1
        for (int k = 0; k < NBAR; k++)
          __syncthreads();
        return;
      }
      const int t = opaque((int)threadIdx.x);
      const int pr = t % BP, i = (t / BP) % T, ba = 2 * pr;
      const int xa = xb * B + ba;
      const float2* hsb = hs + (size_t)blockIdx.x * 16 * WG;
      const int ha = (i * B + ba) * 16;  // round 0's thread (i, ba) wrote its pairs at byte 16 * (i B + ba)
      CPair v[16];
#pragma unroll
      for (int m = 0; m < 16; m += 2)
      {
        const int y = i + ((m + 8) & 15) * T;  // m even: row y + T holds element m + 1
        const float4 pa = ld4s<kStream>(hsb, ha, (m >> 1) * WG * 16);
        const float4 pb = ld4s<kStream>(hsb, ha + 16, (m >> 1) * WG * 16);
        const float ia0 = make_kvec(xa, y, dim, f.dk).inv, ib0 = make_kvec(xa + 1, y, dim, f.dk).inv;
        const float ia1 = make_kvec(xa, y + T, dim, f.dk).inv, ib1 = make_kvec(xa + 1, y + T, dim, f.dk).inv;
        v[m] = CPair{f2v{ia0 * pa.x, ib0 * pb.x}, f2v{ia0 * pa.y, ib0 * pb.y}};
        v[m + 1] = CPair{f2v{ia1 * pa.z, ib1 * pb.z}, f2v{ia1 * pa.w, ib1 * pb.w}};
      }
      fft_run<LOGN, BP, true>(v, i, pr, xch, tw);
#pragma unroll
      for (int m = 0; m < 16; m++)
      {
        const float4 cc = make_float4(v[m].re.x, v[m].im.x, v[m].re.y, v[m].im.y);  // gc of columns ba, ba + 1
        if constexpr (SLAB)
        {
          const size_t part = (size_t)fp.cascades * hsl.S * hsl.w * B;
          const int q = (m * T) / hsl.w, yl0 = (m * T) % hsl.w;
          const size_t el = (((size_t)c * hsl.S + s) * hsl.w + yl0) * B;
          unsigned char* blk = send + sopaque((size_t)q * (part * 40 + (size_t)fp.cascades * 2 * N * 16));
          st4<SA>(blk + part * 32 + el * 8, (i * B + ba) * 8, cc);
        }
        else if constexpr (RG == 1 && RGC == 1)
          st4s<SA>(gc + gbase, (i * B + ba) * 8, m * T * B * 8, cc);
        else
          st4s<SA>(gc + cgbase, half_group_offset<LOGN, RGC>(i, 0, ba) * 8, half_group_offset<LOGN, RGC>(m * T, 0) * 8, cc);
      }
    };
    if constexpr (RSPLIT)
      run_round(slot % 3);
    else if constexpr (HS && PC)
    {
      run_round(0);
      run_round(1);
      run_round_c();
    }
    else if constexpr (HS)
    {
#pragma unroll
      for (int round = 0; round < 3; round++)  // specialised per round: 113 VGPRs, no spills
        run_round(round);
    }
    else
    {
#pragma unroll 1
      for (int round = 0; round < 3; round++)
        run_round(round);
    }
  }
  if constexpr (NYQ)
    if ((HALVES > 1 ? xcd_pair_slot(blockIdx.x, gridDim.x) : (int)blockIdx.x) == (int)gridDim.x - 1)
      for (int idx = threadIdx.x; idx < fp.cascades * N; idx += WG)
        half_nyquist_texel(fp, N, HB, h0, reinterpret_cast<float4*>(send), nullptr, 1, 0, seed, nullptr, 0, idx);
}

}  // namespace oceanfft
