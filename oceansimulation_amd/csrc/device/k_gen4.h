// device/k_gen4.h — the slab-capable four-step column pass (N = 8192 / 16384) and the strip-dealt
// path's transpose of received fields to row-major.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ocean_internal.h"
#include "device/evolve.h"
#include "device/fft.h"
#include "device/grid.h"
#include "device/memory.h"

namespace oceanfft
{

// ------------------------------------------------------------------------------------------------
// Four-step half-spectrum column pass (N = 8192 / 16384; whole grids and slabs of P <= 16 ranks),
// like the standalone EncodeIFFT's (k_cols4_step1/2): no work item holds a 256-KiB column and nothing
// is transposed afterwards. A rank transforms its kept columns u' in [u0, u0 + cols) (x = N/2 + u')
// and, on rank P - 1, the Nyquist column u = -N/2 (x = 0) as local column `cols` (Gen4Geom). With
// y index q = N2 n1 + n2 (q the fftShifted row), each field F becomes
// sum_n2 W_N2^(n2 k2) [W_N^(n2 k1) sum_n1 F(N2 n1 + n2) W_16^(n1 k1)] at output row k1 + 16 k2.
//   step 1 (k_gen4_step1): per (local column, n2): evolve H at the 16 rows N2 ((n1 + 8) mod 16) + n2
//     from h0 (blocked 64 columns wide: one 1-KiB row piece per wave load), then for the three field
//     rounds (A, B), (D, E) and C: the 16-point DFT in registers, times W_N^(n2 k1), into the rank's
//     parts at row N2 k1 + n2 ([c][N][lp], 1-KiB pieces). No LDS exchange.
//   step 2 (k_gen4_step2): per (c, k1, strip of CI local columns): the N2-point FFT along the parts'
//     contiguous rows N2 k1 + n2, written to output row k1 + 16 k2 in DESTINATION-BLOCK order: block
//     q = (k1 + 16 k2) / w, row (k1 + 16 k2) - q w, [c][w][lp] (128-B pieces). This is the all-to-all's
//     send layout, so after the exchange the row pass reads each row's columns from the P source
//     blocks as P contiguous runs (RowSrc) and no transpose pass exists (the strip-dealt path's
//     k_half_to_rows moved 40 B per point).
// Bytes per grid point: h0 8 + parts 20 | parts 20 + blocks 20 | row pass 56 = 124; the exchange
// moves the blocks' 20 B per point.
// ------------------------------------------------------------------------------------------------
constexpr int kGen4Block = 64;  // h0 strip width on this path

template <int LOGN, int MINW = 1>
__global__ __launch_bounds__(256, MINW) void k_gen4_step1(FrameParams fp, Gen4Geom g, const float4* __restrict__ h0,
                                                          unsigned char* __restrict__ parts,
                                                          const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  constexpr int N = S::N, N2 = N / 16;
  __shared__ float2 tw[S::TW_ENTRIES];
  load_twiddles<LOGN>(tw, tw_glob);
  const int lp = g.lp, ncols = g.cols + g.nyq, XB = (ncols + 63) / 64;
  const size_t part = (size_t)fp.cascades * N * lp;  // texels per part
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
    const int ul = xbk * 64 + lane;  // local column
    const bool live = ul < ncols;
    // the Nyquist column is the only live lane of the last wave of rank P - 1 (cols % 64 == 0)
    const bool nyqwave = g.nyq && xbk * 64 == g.cols;
    const int lc = nyqwave ? 0 : lane;
    const int x = nyqwave ? 0 : N / 2 + g.u0 + ul;
    const CascadeFrame f = fp.c[c];
    // one descriptor for the item's 64-column h0 block (uniform per wave)
    const float4* src = h0 + c * g.h0_cstride + (nyqwave ? g.h0_nyq : g.h0_reg + (size_t)xbk * N * kGen4Block);
    const int loff = (n2 * kGen4Block + lc) * 16;
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
    const size_t cb = (size_t)c * N * lp;
    const int soff = (n2 * lp + ul) * 16;
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
      float4* d1 = d0 + (size_t)8 * N2 * lp;
      if (live)
#pragma unroll
        for (int k1 = 0; k1 < 16; k1++)
          st4s<kStream>(k1 < 8 ? d0 : d1, soff, (k1 & 7) * N2 * lp * 16, pair_raw(v[k1]));
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
          st2s<kStream>(d0, soff / 2, k1 * N2 * lp * 8, w[k1]);
    }
  }
}

// Step 2 on one part: per (cascade, k1, strip of CI columns) the N2-point FFT along rows N2 k1 + n2
// of `work` ([c][N][pitch], texels of 16 B), out to destination-block order: output row k1 + 16 k2
// goes to block q = k2 / (N2 / P) at row k1 + 16 (k2 - q N2 / P) of [c][w][pitch], byte offset
// part_off inside the block. T divides N2 / P (P <= 16), so q and the row base are uniform per
// output element m. PAIRS: the texels are split-plane CPairs (gab, gde: raw_pair / pair_raw);
// otherwise two adjacent float2 columns of gc in the reference's (re0, im0, re1, im1) order,
// transformed as the two lanes of one CPair. cols: columns to transform (< pitch).
// CI: columns per workgroup (8: 128-B pieces, 512-thread workgroups, two per CU at N2 = 1024).
// PUT (the one-sided exchange, ocean_peers): block q goes straight to dst[q], the address of this
// rank's block in rank q's receive slot (a peer mapping over xGMI, or local memory for q == rank),
// instead of send + q * blk_bytes; no send buffer exists. (The ready signal after the kernel writes
// back every XCD's L2 before it raises the peers' flags: k_peer_signal_release.)
template <int LOGN2, bool PAIRS, int CI = ColCfg<LOGN2>::C, bool PUT = false>
__global__ __launch_bounds__(FftShape<LOGN2>::T * CI, CI < ColCfg<LOGN2>::C ? 4 : 1) void k_gen4_step2(
    int cascades, int cols, int pitch, const float4* __restrict__ work, unsigned char* __restrict__ send,
    size_t part_off, Gen4Geom g, const float2* __restrict__ tw_glob, const uint64_t* __restrict__ dst)
{
  using S = FftShape<LOGN2>;
  constexpr int N2 = S::N, T = S::T, C = CI, N = N2 * 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN2>(tw, tw_glob);
  const int c0 = threadIdx.x % C, i0 = threadIdx.x / C;
  const int strips = (cols + C - 1) / C;
  const int total = cascades * 16 * strips;
  const int kpb = N2 / g.ranks;  // k2 values per destination block
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    const int cc = opaque(c0), i = opaque(i0);
    const int strip = item % strips, rest = item / strips, k1 = rest & 15, c = rest >> 4;
    const int u = strip * C + cc;
    const bool live = u < cols;
    const float4* src = work + ((size_t)c * N + (size_t)N2 * k1) * pitch;
    const int loff = (i * pitch + (live ? u : cols - 1)) * 16;
    CPair v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
    {
      const float4 r = ld4s<kStream>(src, loff, m * T * pitch * 16);
      v[m] = PAIRS ? raw_pair(r) : to_pair(r);
    }
    fft_run<LOGN2, C, true>(v, i, cc, xch, tw);
    // columns past `cols` get an offset past the descriptor's range: the store is dropped (no branch)
    const int soff = live ? (16 * i * pitch + u) * 16 : kAllBytes;
#pragma unroll
    for (int m = 0; m < 16; m++)
    {
      const int q = (m * T) / kpb, k2b = m * T - q * kpb;
      // the block row base is built at its store (sopaque): hoisted, the 16 bases take 32 SGPRs
      const size_t boff = part_off + ((size_t)c * g.w + k1 + 16 * k2b) * pitch * 16;
      unsigned char* d = PUT ? reinterpret_cast<unsigned char*>(sopaque((size_t)dst[q] + boff))
                             : send + sopaque(q * g.blk_bytes + boff);
      st4<kStream>(d, soff, PAIRS ? pair_raw(v[m]) : from_pair(v[m]));
    }
  }
}

// Strip-dealt half-spectrum fields -> row-major (HalfSlab blocks -> [c][yl][kp], kp = STRIPS * B):
// the received blocks hold, per source rank r, its strips' w rows as [sl][yl][B] runs; the row pass
// wants each row's kept columns u' = strip * B + b contiguous. 256 columns x 16 rows per tile
// through LDS: reads are 16 B-texel runs (one per strip), writes 256-texel (4 KiB for float4) row
// runs, both non-temporal. Measured at N = 16384, float4 (tools/microbench/transbench,
// profiles/r02_transbench.log): 0.955 -> 0.870 ms per part against the earlier 128 x 32 tile with
// default-policy access; the write run length sets the rate (64 x 64: 4.0 TB/s, 128 x 32: 4.5,
// 256 x 16 with nt: 5.0), and strip-stride padding changes nothing.
// E = float4 (gab, gde) or float2 (gc); part_byte_off = the part's offset inside a block.
template <typename E>
__device__ __forceinline__ E ld_nt(const E* p)
{
  if constexpr (sizeof(E) == 16)
  {
    const f4v t = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
    return E{t.x, t.y, t.z, t.w};
  }
  else
  {
    const f2v t = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(p));
    return E{t.x, t.y};
  }
}

template <typename E>
__device__ __forceinline__ void st_nt(E* p, E v)
{
  if constexpr (sizeof(E) == 16)
    __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(p));
  else
    __builtin_nontemporal_store(f2v{v.x, v.y}, reinterpret_cast<f2v*>(p));
}

constexpr int kHalfToRowsTU = 256, kHalfToRowsTY = 16;

template <typename E, int B>
__global__ __launch_bounds__(256) void k_half_to_rows(int cascades, int n, HalfSlab hsl,
                                                      const unsigned char* __restrict__ in, size_t part_byte_off,
                                                      size_t block_bytes, E* __restrict__ out)
{
  constexpr int TU = kHalfToRowsTU, TY = kHalfToRowsTY, PER = TU * TY / 256;
  static_assert(PER == 16 && TU % B == 0, "16 elements per thread");
  __shared__ E tile[TU][TY + 1];
  const int strips = n / (2 * B) + 1, kp = strips * B;
  // tiles never straddle two source blocks: (c, source rank r, column tile within r's strips, row tile)
  const int ranks = (strips + hsl.S - 1) / hsl.S;
  const int tiles_r = (hsl.S * B + TU - 1) / TU, tiles_y = hsl.w / TY;
  const int total = cascades * ranks * tiles_r * tiles_y;
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    int t = item;
    const int tr = t % tiles_r;
    t /= tiles_r;
    const int r = t % ranks;
    t /= ranks;
    const int ty = t % tiles_y, c = t / tiles_y;
    const int u0 = r * hsl.S * B + tr * TU;  // the tile's first column u'
    const int ulim = min(kp, (r + 1) * hsl.S * B);
    const E* src = reinterpret_cast<const E*>(in + (size_t)r * block_bytes + part_byte_off) +
                   (((size_t)c * hsl.S + tr * (TU / B)) * hsl.w + ty * TY) * B;
    // read: b fastest, then row, then strip; all loads are issued before the first LDS write
    E v[PER];
#pragma unroll
    for (int k = 0; k < PER; k++)
    {
      const int L = k * 256 + threadIdx.x, b = L % B, row = (L / B) % TY, sti = L / (TY * B);
      // unconditional loads (a guarded load per element serialises them): columns past the rank's
      // strips read the tile's first element instead, and are not stored
      const bool in_range = u0 + sti * B + b < ulim;
      v[k] = ld_nt(src + (in_range ? ((size_t)sti * hsl.w + row) * B + b : 0));
    }
#pragma unroll
    for (int k = 0; k < PER; k++)
    {
      const int L = k * 256 + threadIdx.x, b = L % B, row = (L / B) % TY, sti = L / (TY * B);
      tile[sti * B + b][row] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; k++)
    {
      const int L = k * 256 + threadIdx.x, row = L / TU, col = L % TU;
      if (u0 + col < ulim)
        st_nt(out + ((size_t)c * hsl.w + ty * TY + row) * kp + u0 + col, tile[col][row]);
    }
    __syncthreads();
  }
}

}  // namespace oceanfft
