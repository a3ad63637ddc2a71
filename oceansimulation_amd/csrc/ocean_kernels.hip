// ocean_kernels.hip — gfx950 device code for the ocean hot path:
//   h0(k) JONSWAP seeding -> h(k,t) evolution fused into the column iFFT -> row iFFT + foam,
//   plus the standalone EncodeIFFT, the slab transpose and the surface consumer.
//
// Reference semantics (paths relative to the reference root):
//   spectrum seeding      resources/spectrum.compute:38-172   (generateSpectrum)
//   evolve + packing      resources/spectrum.compute:183-240  (prepareFFT)
//   2D inverse FFT        resources/fft.compute:21-88 driven by src/FFTCalculator.cpp:73-114
//                         == N^2 * ifft2(ifftshift(X)) per complex lane, no normalisation
//   Jacobian / foam       resources/spectrum.compute:246-259
//
// MI355X design (DESIGN.md has the byte accounting):
//   * Generator frame = 2 HBM passes, column pass first (116 B per height-field point):
//     k_cols_evolve reads the strip-blocked h0 (16 B), evolves and packs both images in registers,
//     iFFTs along y and writes the blocked intermediate (32 B); k_rows_final reads it in 256-B runs
//     (32 B), iFFTs along x and writes the row-major maps (32 B) and the Jacobian (4 B).
//   * Each 1D transform is a self-sorting Stockham FFT held in VGPRs (device/fft.h): 16 points per
//     thread, radix-16 stages, split-plane packed complex math, LDS only between stages. fftShift
//     is folded into load indices; no bit-reversal pass exists.
//   * Persistent grids sized from occupancy (optionally for a CU budget); every loop has a plain
//     item-count exit.
// Device building blocks live in device/{spectrum,memory,fft,evolve}.h; this file holds the kernels
// and their host launchers (ocean_internal.h declares the launchers).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <mutex>
#include <vector>

#include "ocean_internal.h"
#include "device/evolve.h"
#include "device/fft.h"
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
    int rows, float4* __restrict__ images, const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  using R = RowCfg<LOGN>;
  constexpr int N = S::N, T = S::T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN>(tw, tw_glob);

  const int rho0 = threadIdx.x / T, i0 = threadIdx.x % T;
  const int total = rows;  // rows of N packed texels, contiguous (n_images * N for whole images)
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
// Generalisation: GROUP consecutive work slots on blocks b, b+8, ..., b+8(GROUP-1) (one XCD).
template <int GROUP>
__device__ __forceinline__ int xcd_group_slot(int b, int G)
{
  if (G % (8 * GROUP) != 0)
    return b;
  const int xcd = b & 7, j = b >> 3;
  const int grp = xcd * (G / (8 * GROUP)) + j / GROUP;
  return GROUP * grp + j % GROUP;
}

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
            a[m] = ld4s<LA>(src, voff, ((m + 8) & 15) * T * B * 16);  // fftShift on y folded into the load
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
// LA: default-policy loads. Each 128-B line is read half by this block and half by the block of
// the adjacent strip (same XCD, same time); streamed (nt) loads lost the line before the partner's
// read: 1.38 -> 1.12 ms per 8 images (tools/microbench/ifftbench; grouping 4 or 8 strips: no gain).
template <int LOGN, int LA = 0, int GROUP = 2>
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
  for (int item = xcd_group_slot<GROUP>(blockIdx.x, gridDim.x); item < total; item += gridDim.x)
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
      v[m] = to_pair(ld4<LA>(src + ((size_t)(((m + 8) & 15) * T) << LOGN), voff));  // fftShift on y
    fft_run<LOGN, K::C1, true>(v, i, b, xch, tw);
    float4* dst = work + ((size_t)img << (2 * LOGN)) + (size_t)xb * N * B;
    const int soff = (i * B + b) * 16;
#pragma unroll
    for (int m = 0; m < 16; m++)
      st4<kStream>(dst + m * T * B, soff, pair_raw(v[m]));
  }
}

// Standalone EncodeIFFT at N >= 8192: the column transform in four steps (N = 16 N2), so that no
// access is a 16- or 32-byte column piece (one 16384-row column is 256 KiB: an in-place column
// item holds one or two columns and reads 16-32-B pieces, 1.3-2.8 TB/s). For y index n = N2 n1 + n2
// and k = k1 + 16 k2:  X[k1 + 16 k2] = sum_n2 W_N2^(n2 k2) [W_N^(n2 k1) sum_n1 x[N2 n1 + n2] W_16^(n1 k1)].
// Step 1 (this kernel), per (column x, n2): the 16-point inverse DFT over rows N2 n1 + n2 (fftShift
// on y folded into n1: row (n + N/2) mod N = N2 ((n1 + 8) mod 16) + n2), times W_N^(n2 k1), into the
// work slab at row N2 k1 + n2, split planes. Lanes run along x: every load and store of a wave is one
// 1-KiB row piece, and there is no LDS exchange. The work slab holds columns [x0, x0 + wc).
template <int LOGN>
__global__ __launch_bounds__(256) void k_cols4_step1(int images, int x0, int wc, const float4* __restrict__ img,
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
    const int xl = xbk * 64 + lane;  // column within the slab
    const float4* src = img + ((size_t)im << (2 * LOGN)) + x0 + xl;
    CPair v[16];
#pragma unroll
    for (int n1 = 0; n1 < 16; n1++)
    {
      const f4v r = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(src + (size_t)(N2 * ((n1 + 8) & 15) + n2) * N));
      v[n1] = to_pair(make_float4(r.x, r.y, r.z, r.w));
    }
    idft16(v);
    apply_stage_twiddles<LOGN>(v, n2, tw);  // v[k1] *= W_N^(n2 k1)
    float4* dst = work + (size_t)im * N * wc + xl;
#pragma unroll
    for (int k1 = 0; k1 < 16; k1++)
    {
      const float4 o = pair_raw(v[k1]);
      __builtin_nontemporal_store(f4v{o.x, o.y, o.z, o.w}, reinterpret_cast<f4v*>(dst + (size_t)(N2 * k1 + n2) * wc));
    }
  }
}

// Step 2, per (image, k1, strip of C slab columns): the N2-point inverse FFT along the work slab's
// contiguous rows N2 k1 + n2 (n2 = i + m T), output X[k1 + 16 k2] to image row k1 + 16 k2 in the
// reference layout. Loads and stores are C * 16 = 256-byte row pieces. tw_glob: the N2-point table.
template <int LOGN2>
__global__ __launch_bounds__(ColCfg<LOGN2>::WG) void k_cols4_step2(int images, int x0, int wc,
                                                                 const float4* __restrict__ work, float4* __restrict__ img,
                                                                 const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN2>;
  using K = ColCfg<LOGN2>;
  constexpr int N2 = S::N, T = S::T, C = K::C, LOGN = LOGN2 + 4, N = N2 * 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  load_twiddles<LOGN2>(tw, tw_glob);
  const int c0 = threadIdx.x % C, i0 = threadIdx.x / C;
  const int strips = wc / C;
  const int total = images * 16 * strips;
  for (int item = blockIdx.x; item < total; item += gridDim.x)
  {
    const int c = opaque(c0), i = opaque(i0);
    const int strip = item % strips, rest = item / strips, k1 = rest & 15, im = rest >> 4;
    const int xl = strip * C + c;
    const float4* src = work + (size_t)im * N * wc + (size_t)N2 * k1 * wc + xl;
    CPair v[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
    {
      const f4v r = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(src + (size_t)(i + m * T) * wc));
      v[m] = raw_pair(make_float4(r.x, r.y, r.z, r.w));
    }
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
// One h0 texel evaluated in place: (h0(k), conj(h0(-k))), -k at index N - i
// (spectrum.compute:160-168), with the evaluator and arguments of k_generate_spectrum(_pairs).
__device__ __forceinline__ float4 seed_texel(const SpectrumConsts& q, int x, int y, float dim)
{
  const float2 a = spectrum_amplitude(q, (float)x, (float)y);
  const float2 c = spectrum_amplitude(q, dim - (float)x, dim - (float)y);
  return make_float4(a.x, a.y, c.x, -c.y);
}

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
// 2p, 2p + 1 on one XCD, whose loads share h0 lines and whose half-line stores meet in L2).
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
template <int LOGN, int LA = 0, int SA = kStream, bool HS = false, bool SLAB = false, bool SEED = false, int RG = 1,
          int RGC = 1, int CPI = ColFirstCfg<LOGN>::B, bool HP = false, bool PC = false, int HL = 0, int HK = 0>
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
  static_assert(CPI * HALVES == B && HALVES <= 2 && (HALVES == 1 || (!SLAB && !SEED)), "whole or half strips");
  static_assert((HL == 0 && HK == 0) || (HS && HP && !PC && HL + HK <= 8), "H pairs outside the scratch");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  void* xch = smem + ((S::TW_ENTRIES * 8 + 15) / 16) * 16;
  float4* hlds = reinterpret_cast<float4*>(static_cast<unsigned char*>(xch) + K::LDS1);  // HL pairs [p][thread]
  load_twiddles<LOGN>(tw, tw_glob);

  const int nstrips = SLAB ? hsl.nstrips : STRIPS;
  const int total = fp.cascades * nstrips * HALVES;
  const float dim = (float)N;
  for (int item = HALVES > 1 ? xcd_pair_slot(blockIdx.x, gridDim.x) : blockIdx.x; item < total; item += gridDim.x)
  {
    const int hh = HALVES > 1 ? item % HALVES : 0, si = HALVES > 1 ? item / HALVES : item;
    const int c = si / nstrips, s = si - c * nstrips;  // s: the rank's strip index
    const int sg = SLAB ? hsl.strip0 + s : s;           // global strip
    if (HALVES > 1 && sg == STRIPS - 1 && hh != 0)
      continue;  // Nyquist strip: only column 0 (u = -N/2) is kept (uniform per workgroup)
    const int b = opaque((int)threadIdx.x) % CPI + hh * CPI;  // column within the strip
    const int xb = sg == STRIPS - 1 ? 0 : N / (2 * B) + sg;
    const CascadeFrame f = fp.c[c];
    const float4* src = (!SLAB || h0_full) ? h0 + ((size_t)c * (N / B) + xb) * N * B
                                           : h0 + ((size_t)c * nstrips + s) * N * B;
    // the strip's first texel in the cascade's fields (whole grids); + half_group_offset(m T, 0) per m
    const size_t gbase = RG == 1 ? ((size_t)c * STRIPS + s) * N * B
                                 : (size_t)c * STRIPS * N * B + half_group_offset<LOGN, RG>(0, s);
    const size_t cgbase = RGC == 1 ? ((size_t)c * STRIPS + s) * N * B
                                   : (size_t)c * STRIPS * N * B + half_group_offset<LOGN, RGC>(0, s);
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
#pragma unroll
        for (int m = 0; m < 16; m++)  // fftShift on y folded into the load
          a[m] = ld4s<LA>(src, voff, ((m + 8) & 15) * T * B * 16);
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
      fft_run<LOGN, CPI, true>(v, i, HALVES > 1 ? opaque((int)threadIdx.x) % CPI : b, xch, tw);
#pragma unroll
      for (int m = 0; m < 16; m++)
      {
        if constexpr (SLAB)
        {
          // row y = m T + i lies in block q = m T / w (w is a multiple of T), at yl = m T % w + i
          const size_t part = (size_t)fp.cascades * hsl.S * hsl.w * B;  // elements per part
          const int q = (m * T) / hsl.w, yl0 = (m * T) % hsl.w;
          const size_t el = (((size_t)c * hsl.S + s) * hsl.w + yl0) * B;
          // block = the three parts, then the Nyquist-row term [c][2][N] (half_slab_block_bytes).
          // The block base is built at its store (sopaque): hoisted, the 16 descriptors spilled SGPRs.
          unsigned char* blk = send + sopaque((size_t)q * (part * 40 + (size_t)fp.cascades * 2 * N * 16));
          if (round == 0)
            st4<SA>(blk + el * 16, voff, pair_raw(v[m]));
          else if (round == 1)
            st4<SA>(blk + part * 16 + el * 16, voff, pair_raw(v[m]));
          else
            st2<SA>(blk + part * 32 + el * 8, (i * B + b) * 8, make_float2(v[m].re.x, v[m].im.x));
        }
        else if constexpr (RG == 1 && RGC == 1)
        {
          if (round == 0)
            st4s<SA>(gab + gbase, voff, m * T * B * 16, pair_raw(v[m]));
          else if (round == 1)
            st4s<SA>(gde + gbase, voff, m * T * B * 16, pair_raw(v[m]));
          else
            st2s<SA>(gc + gbase, (i * B + b) * 8, m * T * B * 8, make_float2(v[m].re.x, v[m].im.x));
        }
        else if (round == 0)  // one descriptor per field; the row group of m T in soffset
          st4s<SA>(gab + gbase, half_group_offset<LOGN, RG>(i, 0, b) * 16, half_group_offset<LOGN, RG>(m * T, 0) * 16,
                   pair_raw(v[m]));
        else if (round == 1)
          st4s<SA>(gde + gbase, half_group_offset<LOGN, RG>(i, 0, b) * 16, half_group_offset<LOGN, RG>(m * T, 0) * 16,
                   pair_raw(v[m]));
        else
          st2s<SA>(gc + cgbase, half_group_offset<LOGN, RGC>(i, 0, b) * 8, half_group_offset<LOGN, RGC>(m * T, 0) * 8,
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
    if constexpr (HS && PC)
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
}

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

// The Nyquist-row term: for u = -u' (0 < u' < N/2) the pass-2 rebuild s_F conj(G_F(q, u')) misses
// (-1)^q Delta_F(u'), Delta_F(u') = F(-N/2, -u') - s_F conj(F(-N/2, u')). Its lanes (the kx
// factors of pass 2 applied to Delta) form one row spectrum per image, spec[c][img][x] (zero
// outside 0 < x < N/2); pass 2 adds (-1)^q spec to the lanes it rebuilds at u < 0.
// h0row (slabs, whose h0 holds only their strips): the row y = 0 texels of every column, [c][x].
// copies / copy_stride: the strip-dealt path writes the term into every destination block of the
// exchange buffer, so each frame's row pass reads the term of its own frame (the pipeline keeps two
// frames in flight).
// seed (the fused re-seed frame, h0 not materialised): the two row-0 texels are evaluated here.
__global__ __launch_bounds__(256) void k_half_nyquist(FrameParams fp, int n, int blk, const float4* __restrict__ h0,
                                                      float4* __restrict__ spec, const float4* __restrict__ h0row,
                                                      int copies, size_t copy_stride,
                                                      const SpectrumConsts* __restrict__ seed)
{
  const int total = fp.cascades * n;
  const float dim = (float)n;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x)
  {
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
      float4* sp = reinterpret_cast<float4*>(reinterpret_cast<unsigned char*>(spec) + k * copy_stride);
      sp[((size_t)c * 2 + 0) * n + x] = s01;
      sp[((size_t)c * 2 + 1) * n + x] = s23;
    }
  }
}

// Pass 2: RPW rows of one image. Element m of the x transform is column x = ((m + 8) & 15) T + i,
// u = x - N/2: m < 8 -> u = m T + i >= 0 (stored column u), m >= 8 -> u < 0. Every thread loads
// only its 8 direct elements (and thread 0 the Nyquist column for m = 8) and computes the lanes
// both at u (its own) and at -u, adding there the Nyquist-row term (-1)^y S(-u); the -u lanes go
// through LDS to the thread that holds -u: element 15 - m of thread T - i (thread 0: element
// 16 - m of itself). Each stored value is read once from HBM. Then the x-iFFT, maps + Jacobian.
// ABL (tools/microbench timing ablations, results wrong by construction): 1 = no HBM loads,
// 2 = no x transform, 3 = no mirror exchange through LDS.
// RPW_ = 2 (default): 512-thread workgroups, two per CU, so one workgroup's loads overlap the
// other's transform (the LDS mirror exchange adds a barrier the 1024-thread, one-per-CU shape cannot
// hide: 1.92 -> 1.69 ms at 8 x 4096^2, tools/microbench/genbench).
// BOTH: one item = both images of its rows (image 0, then image 1), so C is loaded once and kept
// in VGPRs (16) for image 1 instead of being fetched again by a second item.
// RM (strip-dealt path, after k_half_to_rows): the fields are row-major [c][rows][kp], column u' = u
// for u in [0, N/2] (u' = N/2: the Nyquist column), and the pass covers `rows` rows (a slab's w).
// RG / RGC (whole grids): the field layout pass 1 wrote (half_group_offset).
// FB: the field strips' width (half_group_offset); GRP: consecutive items run together on one XCD
// (2: pairs, xcd_pair_slot; 4: FB = 2 with RGC = 8, where four items share each gc line).
// XS (RPW = 1, N = 16 T, T = 1024: one row per 16-wave workgroup): the x transform in four steps
// so that most of it runs between workgroup barriers instead of across them. With n = n1 + 16 n2
// and k = k2 + T k1: a transposition through LDS (T_in, which also does the mirror exchange's job)
// gives wave n1 the T inputs x(n1 + 16 n2); each wave runs its T-point sub-transform (fft_run<LOGN -
// 4>, 64 lanes x 16 points) in its own LDS region, ordered by the LDS's in-order execution of one
// wave's instructions instead of barriers; twiddles W_N^(n1 k2); a second transposition (T_out)
// gives thread k2 the 16 values over n1, and a 16-point DFT in registers leaves X(k2 + T k1) in the
// plain path's layout (coalesced stores). Barriers per image: 7 instead of 14 (mirror 2 + three
// exchanges of two halves x 2 + 1). rm16bench priced the barriers of the 16384 pass at ~1 ms of
// 3.8. tw2_glob: the T-point table (appended for 8192/16384 by ocean_fft_create).
template <int LOGN>
struct XsCfg
{
  static constexpr int L2 = LOGN - 4;
  // region of one n1 (slots of 8 B): holds a sub-transform's padded exchange (PADDED + 4), and
  // RS = 1 mod 16 spreads T_in's 16-lane writes (16 regions at once) over all 32 banks
  static constexpr int RS = ((FftShape<L2>::PADDED + 4 + 14) / 16) * 16 + 1;
  static constexpr int TW1 = ((FftShape<LOGN>::TW_ENTRIES * 8 + 15) / 16) * 16;
  static constexpr int TW2 = ((FftShape<L2>::TW_ENTRIES * 8 + 15) / 16) * 16;
  static constexpr int LDS = TW1 + TW2 + 16 * RS * 8;
};

template <int LOGN, int LA = kStream, int SA = kStream, int ABL = 0, int RPW_ = 2, bool BOTH = false, bool RM = false,
          int RG = 1, int RGC = 1, int FB = 4, int GRP = 2, bool IL = true, bool XS = false>
__global__ __launch_bounds__(FftShape<LOGN>::T * RPW_) void k_rows_half(
    FrameParams fp, const float4* __restrict__ gab, const float4* __restrict__ gde, const float2* __restrict__ gc,
    const float4* __restrict__ spec, float4* __restrict__ maps, float* __restrict__ jac, FoamParams foam,
    const float2* __restrict__ tw_glob, int rows, int kp, const float2* __restrict__ tw2_glob)
{
  using S = FftShape<LOGN>;
  using K = ColFirstCfg<LOGN>;
  using HC = HalfCfg<LOGN>;
  constexpr int N = S::N, T = S::T, B = K::B, RPW = RPW_, STRIPS = HC::STRIPS, WG = T * RPW;
  static_assert(WG * 8 * 16 <= lds_row_slots<LOGN>(RPW) * 8, "mirror exchange fits the transform's LDS");
  static_assert(!XS || (RPW == 1 && T == 1024), "XS: one 16-wave row per workgroup");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float2* tw = reinterpret_cast<float2*>(smem);
  float2* tw2 = reinterpret_cast<float2*>(smem + XsCfg<LOGN>::TW1);
  void* xch = smem + (XS ? XsCfg<LOGN>::TW1 + XsCfg<LOGN>::TW2 : ((S::TW_ENTRIES * 8 + 15) / 16) * 16);
  CPair* mir = reinterpret_cast<CPair*>(xch);  // [m < 8][thread]: lanes at -u for the partner
  if constexpr (XS)
  {
    for (int e = threadIdx.x; e < FftShape<XsCfg<LOGN>::L2>::TW_ENTRIES; e += blockDim.x)
      tw2[e] = tw2_glob[e];
  }
  load_twiddles<LOGN>(tw, tw_glob);

  const int blocks = (RM ? rows : N) / RPW;
  const int b0 = threadIdx.x % B, r0 = (threadIdx.x / B) % RPW, ihi0 = threadIdx.x / (B * RPW);
  // After the first exchange: RPW = 2 interleaves the two rows (lanes: row fastest) and their LDS
  // regions (CI = 2, slot = 2 pa + row), so a wave's reads of 32 consecutive positions never straddle
  // a pad slot: conflict-free exchanges at 4096 (the row layout cost one extra cycle per 32-lane read
  // group, 262 K LDS cycles per CU per frame = SQ_LDS_BANK_CONFLICT; tools/lds_banks.py models both).
  // (A/B, halfbench rows: 1.449 -> 1.417 ms at 8 x 4096^2, 0.341 -> 0.335 at 2048; at 1024 the row
  // layout stays: 0.079 vs 0.083 ms). IL = false: the row layout.
  constexpr int CI = (IL && RPW == 2 && T >= 128) ? 2 : 0;
  const int i20 = CI ? (threadIdx.x / RPW) % T : threadIdx.x % T, r20 = CI ? threadIdx.x % RPW : threadIdx.x / T;
  const int total = fp.cascades * (BOTH ? 1 : 2) * blocks;
  const float dim = (float)N;
  // RPW = 2: C's row pairs are 64-B halves of 128-B lines; items 2p, 2p+1 (the same line) run
  // together on one XCD so the line is fetched once
  // (RPW = 1 with GRP = 4, an A/B: the 4 rows of a gc line on one XCD)
  for (int item = RPW != 2 && GRP != 4 ? blockIdx.x : GRP == 4 ? xcd_group_slot<4>(blockIdx.x, gridDim.x)
                                                                : xcd_pair_slot(blockIdx.x, gridDim.x);
       item < total; item += gridDim.x)
  {
    const int cimg0 = item / blocks, y0 = (item - cimg0 * blocks) * RPW;
    float2 ckeep[8];  // BOTH: image 0's C loads, reused by image 1
    float2 cnyq;
#pragma unroll
    for (int pass = 0; pass < (BOTH ? 2 : 1); pass++)
    {
    const int cimg = BOTH ? cimg0 * 2 + pass : cimg0;
    const int b = opaque(b0), ihi = opaque(ihi0), r = RPW == 1 ? 0 : opaque(r0);
    const int i = ihi * B + b;
    const int c = cimg >> 1, img = BOTH ? pass : (cimg & 1);
    const float dk = fp.c[c].dk;
    // RM: the item's first row; element (r, u) at r kp + u
    const size_t base = RM ? ((size_t)c * rows + y0) * kp : (size_t)c * STRIPS * N * B;
    const int y = y0 + r;
    const float sgy = (y & 1) ? -1.0f : 1.0f;  // (-1)^q of the Nyquist-row term
    const float4* sp = spec + (size_t)cimg * N;
    const int tid = opaque((int)threadIdx.x);
    CPair v[16];  // XS: own lanes in v[m], the -u lanes in v[m + 8] until the transposition
#pragma unroll
    for (int m = 0; m < 8; m++)
    {
      const int u = m * T + i;               // >= 0, column x = N/2 + u
      const int off = RM ? r * kp + u : half_group_offset<LOGN, RG, FB>(y, u / FB, u % FB);
      const int offc = RM ? off : half_group_offset<LOGN, RGC, FB>(y, u / FB, u % FB);
      const float kx = (float)u * dk;        // ((float)x - N/2) dk, x - N/2 exact
      const float4 s4 = ld4<0>(sp, (N / 2 - u) * 16);  // the -u column's Nyquist-row term (x = N/2 - u)
      CPair own, neg;
      if (ABL == 1)
      {
        own = CPair{f2v{kx, s4.x}, f2v{(float)off, sgy}};
        neg = CPair{f2v{s4.y, kx}, f2v{sgy, (float)u}};
      }
      else if (img == 0)
      {
        const CPair p = raw_pair(ld4<LA>(gab + base, off * 16));  // (A, B)
        const float2 cc = ld2<LA>(gc + base, offc * 8);             // C
        if (BOTH)
          ckeep[m] = cc;
        const float Ar = p.re.x, Ai = p.im.x, Br = p.re.y, Bi = p.im.y, Cr = cc.x, Ci = cc.y;
        // at u: lane0 = (1 - kx) A, lane1 = i B - kx C
        own = CPair{f2v{(1.0f - kx) * Ar, -Bi - kx * Cr}, f2v{(1.0f - kx) * Ai, Br - kx * Ci}};
        // at -u (kx -> -kx, A -> conj A, B -> -conj B, C -> conj C): lane0 = (1 + kx) conj A,
        // lane1 = i (-conj B) + kx conj C
        neg = CPair{f2v{(1.0f + kx) * Ar + sgy * s4.x, -Bi + kx * Cr + sgy * s4.z},
                    f2v{-(1.0f + kx) * Ai + sgy * s4.y, -Br - kx * Ci + sgy * s4.w}};
      }
      else
      {
        const CPair q = raw_pair(ld4<LA>(gde + base, off * 16));  // (D, E)
        const float2 cc = BOTH ? ckeep[m] : ld2<LA>(gc + base, offc * 8);  // C
        const float Cr = cc.x, Ci = cc.y, Dr = q.re.x, Di = q.im.x, Er = q.re.y, Ei = q.im.y;
        const float kx2 = kx * kx;
        // at u: lane2 = i (D - kx^2 C), lane3 = -E - i kx D
        own = CPair{f2v{-(Di - kx2 * Ci), -Er + kx * Di}, f2v{Dr - kx2 * Cr, -Ei - kx * Dr}};
        // at -u (D -> -conj D, C -> conj C, E -> conj E, kx -> -kx): lane2 = i (-conj D - kx^2 conj C),
        // lane3 = -conj E + i kx (-conj D)
        neg = CPair{f2v{-(Di + kx2 * Ci) + sgy * s4.x, -Er - kx * Di + sgy * s4.z},
                    f2v{-Dr - kx2 * Cr + sgy * s4.y, Ei - kx * Dr + sgy * s4.w}};
      }
      v[m] = own;
      if constexpr (ABL == 3 || XS)
        v[m + 8] = neg;
      else
        mir[m * WG + tid] = neg;
    }
    if constexpr (ABL != 3 && !XS)
      __syncthreads();
    // own elements m >= 8 (u < 0): from the partner's mirror slots; thread 0's m = 8 is the Nyquist
    // column (u = -N/2), read directly
    const int tp = i == 0 ? tid : tid + (((T - i) / B - ihi) * B * RPW) + ((T - i) % B - b);
#pragma unroll
    for (int m = 8; m < 16; m++)
    {
      if (ABL == 3 || ABL == 1)
      {
        if (ABL == 1)
          v[m] = mir[(i == 0 ? 16 - m : 15 - m) * WG + tp];
      }
      else if (i == 0 && m == 8)
      {
        // Nyquist column: first column of the last strip
        const int off = RM ? r * kp + N / 2 : half_group_offset<LOGN, RG, FB>(y, N / 2 / FB);
        const int offc = RM ? off : half_group_offset<LOGN, RGC, FB>(y, N / 2 / FB);
        const float kx = -(dim / 2.0f) * dk;
        float2 cc;
        if (BOTH && img == 1)
          cc = cnyq;
        else
          cc = ld2<LA>(gc + base, offc * 8);  // C
        if (BOTH && img == 0)
          cnyq = cc;
        if (img == 0)
        {
          const CPair p = raw_pair(ld4<LA>(gab + base, off * 16));  // (A, B)
          v[m] = CPair{f2v{(1.0f - kx) * p.re.x, -p.im.y - kx * cc.x},
                       f2v{(1.0f - kx) * p.im.x, p.re.y - kx * cc.y}};
        }
        else
        {
          const CPair q = raw_pair(ld4<LA>(gde + base, off * 16));  // (D, E): D = (re.x, im.x)
          const float kx2 = kx * kx;
          v[m] = CPair{f2v{-(q.im.x - kx2 * cc.y), -q.re.y + kx * q.im.x},
                       f2v{q.re.x - kx2 * cc.x, -q.im.y - kx * q.re.x}};
        }
      }
      else if constexpr (!XS)
        v[m] = mir[(i == 0 ? 16 - m : 15 - m) * WG + tp];
    }
    if constexpr (ABL != 3 && !XS)
      __syncthreads();  // the transform's first exchange reuses the LDS
    int i2 = opaque(i20), r2 = RPW == 1 ? 0 : opaque(r20);
    if constexpr (XS)
    {
      // x index n = n1 + 16 n2, output k = k2 + 1024 k1 (T = 1024): transposition T_in gives wave
      // n1 = w the inputs x(w + 16 n2) (own lanes at n, the -u lanes at N - n, thread 0's Nyquist
      // column at N/2); the wave's 1024-point sub-transform; times W_N^(n1 k2); transposition T_out
      // gives thread k2 = tid the 16 values Z_n1(k2); the 16-point DFT over n1 leaves
      // v[k1] = X(tid + T k1): the plain path's store layout. LDS slot of n: (n mod 16) RS + n / 16.
      constexpr int L2 = XsCfg<LOGN>::L2, RS = XsCfg<LOGN>::RS;
      const int w = tid >> 6, l = tid & 63;
      float2* xs = reinterpret_cast<float2*>(xch);
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
      i2 = tid;
    }
    else if constexpr (ABL != 2)
      fft_run<LOGN, CI, true>(v, i, r, i2, r2, xch, tw);
    float4* dst = maps + ((size_t)cimg * (RM ? rows : N) + y0) * N;
    const int woff = ((r2 << LOGN) + i2) * 16;
#pragma unroll
    for (int m = 0; m < 16; m++)
      st4<SA>(dst + m * T, woff, from_pair(v[m]));
    if (img & 1)
    {
      // displacementMap (Dz, dDx/dx, dDz/dz, dDx/dz) = (re0, im0, re1, im1): Jacobian,
      // spectrum.compute:246-259
      const float lam = foam.displacement[c];
      float* jb = jac + ((size_t)c * (RM ? rows : N) + y0) * N;
      const int joff = ((r2 << LOGN) + i2) * 4;
#pragma unroll
      for (int m = 0; m < 16; m++)
        st1<SA>(jb + m * T, joff,
                (1.0f + lam * v[m].im.x) * (1.0f + lam * v[m].re.y) - lam * lam * v[m].im.y * v[m].im.y);
    }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Whole grids of N = 16384 (one rank): the half-spectrum column pass in four steps, like the
// standalone EncodeIFFT's (k_cols4_step1/2), so that no pass holds a 256-KiB column and nothing is
// transposed afterwards. Kept column u' in [0, kp), kp = N/2 + B (u' < N/2: x = N/2 + u'; then the
// Nyquist strip x = u' - N/2). With y index q = N2 n1 + n2 (q the fftShifted row), each field F
// becomes sum_n2 W_N2^(n2 k2) [W_N^(n2 k1) sum_n1 F(N2 n1 + n2) W_16^(n1 k1)] at output row
// k1 + 16 k2.
//   step 1 (k_gen4_step1): per (u', n2): evolve H at the 16 rows N2 ((n1 + 8) mod 16) + n2 from h0
//     (blocked 64 columns wide, kGen4Block: one 1-KiB row piece per wave load), then for the three
//     field rounds (A, B), (D, E) and C: the 16-point DFT in registers, times W_N^(n2 k1), into the
//     work parts at row N2 k1 + n2 (row-major [c][row][kp], 1-KiB pieces). No LDS exchange.
//   step 2 (k_gen4_step2): per (c, k1, strip of 16 kept columns): the N2-point FFT along the work's
//     contiguous rows N2 k1 + n2, out to the row-major fields rm[c][k1 + 16 k2][u'] the row pass
//     (k_rows_half RM) reads; 256-B (gc: 128-B) pieces.
// Bytes per grid point: h0 8 + parts 20, parts 20 + fields 20, then the row pass 56: 124, as the
// strip-dealt column pass (28) + transposes (40) + rows (56), but without the one-column items.
// ------------------------------------------------------------------------------------------------
constexpr int kGen4Block = 64;  // h0 strip width on this path
// Row pitch (texels) of the work parts and of the row-major fields: kp rounded up to 16 texels, so
// every 16-column strip is whole 128-B lines (kp = N/2 + B is odd at 16384; an odd pitch put every
// 256-B strip piece across three lines: step 2 took 2x as long).
template <int LOGN>
struct Gen4Cfg
{
  static constexpr int N = 1 << LOGN, N2 = N / 16, B = ColFirstCfg<LOGN>::B, KP = N / 2 + B;
  static constexpr int PITCH = (KP + 15) / 16 * 16;
};

template <int LOGN, int MINW = 1>
__global__ __launch_bounds__(256, MINW) void k_gen4_step1(FrameParams fp, const float4* __restrict__ h0,
                                                    unsigned char* __restrict__ parts, const float2* __restrict__ tw_glob)
{
  using S = FftShape<LOGN>;
  using G = Gen4Cfg<LOGN>;
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

// Step 2 on one part: per (cascade, k1, strip of C columns) the N2-point FFT along rows N2 k1 + n2 of
// `work`, out to rows k1 + 16 k2 of `rm`; both [c][N][pitch] in texels of 16 B. PAIRS: the texels
// are split-plane CPairs (gab, gde: raw_pair / pair_raw); otherwise two adjacent float2 columns of gc
// in the reference's (re0, im0, re1, im1) order, transformed as the two lanes of one CPair.
// cols: columns to transform (< pitch). Descriptors: one for the strip's input rows, two for its
// output (rows below and above 16 * 8 T) so the 32-bit offsets stay below 2 GiB.
// CI: columns per workgroup (ColCfg's 16: 256-B pieces, one 1024-thread workgroup per CU at N2 =
// 1024; 8: 128-B pieces, two 512-thread workgroups per CU).
template <int LOGN2, bool PAIRS, int CI = ColCfg<LOGN2>::C>
__global__ __launch_bounds__(FftShape<LOGN2>::T * CI, CI < ColCfg<LOGN2>::C ? 4 : 1) void k_gen4_step2(int cascades, int cols, int pitch,
                                                                 const float4* __restrict__ work, float4* __restrict__ rm,
                                                                 const float2* __restrict__ tw_glob)
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
    float4* d0 = rm + ((size_t)c * N + k1) * pitch;
    float4* d1 = d0 + (size_t)16 * 8 * T * pitch;
    const int soff = (16 * i * pitch + u) * 16;
    if (live)
#pragma unroll
      for (int m = 0; m < 16; m++)
        st4s<kStream>(m < 8 ? d0 : d1, soff, (m & 7) * 16 * T * pitch * 16, PAIRS ? pair_raw(v[m]) : from_pair(v[m]));
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

// Grid sizing. With the whole device available (cus >= the device's CUs) every kernel with an item
// loop gets a one-shot grid, one block per work item: the hardware dispatcher then hands items out
// in order, so the blocks in flight at any time work on neighbouring items (adjacent strips share
// 128-B lines in L2, rows stream through neighbouring DRAM pages). Measured against persistent grids
// (resident blocks x CUs, same kernels; tools/microbench/gridbench, profiles/r02_gridbench.log):
// row pass 1.513 -> 1.453 ms, EncodeIFFT strided pass 1.115 -> 0.927 ms, 16384 column pass 6.69 ->
// 5.56 ms. Under a CU budget (ocean_fft_set_cu_budget: CUs left free for RCCL's copy kernels in
// the slab pipeline) grids stay persistent, so at most `cus` CUs' worth of blocks exist. Kernels
// with per-block scratch (the H scratch of the half-spectrum column pass) cap the grid themselves.
// The occupancy query and the dynamic-LDS attribute are set once per kernel instantiation (host API
// calls cost microseconds; a frame is two launches).
static int device_cu_count()
{
  static const int n = [] {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return c;
  }();
  return n;
}

static bool g_force_persistent = false;  // tools/microbench A/B only (they include this file)

static bool one_shot_grids(int cus)
{
  const int d = device_cu_count();
  return !g_force_persistent && d > 0 && cus >= d;
}

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
  if (one_shot_grids(cus))
    return items < 1 ? 1 : items;
  long g = (long)per_cu * cus;
  if (g > items)
    g = items;
  return g < 1 ? 1 : (int)g;
}

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

bool half_spectrum_supported(int logn) { return logn >= 10 && logn <= 12; }

size_t half_field_texels(int logn)
{
  const size_t n = (size_t)1 << logn;
  return (n / 8 + 1) * n * 4;  // HalfCfg: STRIPS * N * B per cascade (B = 4)
}

bool half_slab_supported(int logn);
size_t half_hs_bytes(int logn, int blocks)
{
  return half_slab_supported(logn) ? (size_t)blocks * 16 * 1024 * sizeof(float2) : 0;  // WG1 <= 1024
}

hipError_t launch_half_columns(int logn, const FrameParams& fp, const float4* h0, float4* gab, float4* gcd, float2* ge,
                               float4* spec, const float2* tw, hipStream_t stream, int cus, float2* hs, int hs_blocks,
                               const void* seed_consts, int variant)
{
  const SpectrumConsts* seed = static_cast<const SpectrumConsts*>(seed_consts);
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (!HalfCfg<LOGN>::SUPPORTED)
      return hipErrorInvalidValue;
    else
    {
      using K = ColFirstCfg<LOGN>;
      using S = FftShape<LOGN>;
      const int n = S::N;
      // the Nyquist-row term: one row spectrum per image, then its x-iFFT (in place)
      long blocks = ((long)fp.cascades * n + 255) / 256;
      if (blocks > (long)cus * 4)
        blocks = (long)cus * 4;
      hipLaunchKernelGGL(k_half_nyquist, dim3((unsigned)blocks), dim3(256), 0, stream, fp, n, K::B, h0, spec,
                         (const float4*)nullptr, 1, (size_t)0, seed);
      hipError_t e = hipGetLastError();
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

hipError_t launch_half_rows(int logn, const FrameParams& fp, const float4* gab, const float4* gcd, const float2* ge,
                            const float4* rcorr, float4* maps, float* jac, const FoamParams& foam, const float2* tw,
                            hipStream_t stream, int cus, int ablation)
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
      const int rpw = ablation == 4 ? R4 : (ablation == 5 || ablation == 16 || (ablation == 0 && ONE_ROW)) ? 1 : 2;
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
                         S::N, 0, (const float2*)nullptr);
      return hipGetLastError();
    }
  });
}

// ---- strip-dealt half-spectrum path (slabs, and whole grids of N = 8192 / 16384) ----
bool half_slab_supported(int logn) { return logn >= 10 && logn <= 14; }

int half_strips(int logn) { return (1 << logn) / (2 * spectrum_block(logn)) + 1; }

// block = gab | gde | gc parts (40 B per element) | the Nyquist-row term [c][2][N] float4
static size_t half_slab_spec_offset(int logn, int cascades, const HalfSlab& h)
{
  return (size_t)40 * cascades * h.S * h.w * spectrum_block(logn);
}

size_t half_slab_block_bytes(int logn, int cascades, const HalfSlab& h)
{
  return half_slab_spec_offset(logn, cascades, h) + (size_t)cascades * 2 * (1 << logn) * sizeof(float4);
}

size_t half_slab_row_texels(int logn, int cascades, int w)
{
  return (size_t)cascades * w * half_strips(logn) * spectrum_block(logn);
}

hipError_t launch_generate_spectrum_row(const OceanSettings& s, int n, float4* row, hipStream_t stream)
{
  // the slab kernel over one row: the same evaluator in the same code, so bit-identical texels
  hipLaunchKernelGGL(k_generate_spectrum, dim3((n + 255) / 256), dim3(256), 0, stream, spectrum_consts(s, n), n, 1, 0,
                     n, row, 1);
  return hipGetLastError();
}

hipError_t launch_half_slab_columns(int logn, const FrameParams& fp, const HalfSlab& hsl, int ranks, const float4* h0,
                                    bool h0_full, const float4* h0row, void* send, const float2* tw,
                                    hipStream_t stream, int cus, float2* hs, int hs_blocks)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (!HalfCfg<LOGN>::SLAB_SUPPORTED)
      return hipErrorInvalidValue;
    else
    {
      using K = ColFirstCfg<LOGN>;
      using S = FftShape<LOGN>;
      const int n = S::N;
      if (hsl.w % S::T != 0 || !hs)
        return hipErrorInvalidValue;
      long blocks = ((long)fp.cascades * n + 255) / 256;
      if (blocks > (long)cus * 4)
        blocks = (long)cus * 4;
      const size_t blk = half_slab_block_bytes(LOGN, fp.cascades, hsl);
      float4* spec = reinterpret_cast<float4*>((unsigned char*)send + half_slab_spec_offset(LOGN, fp.cascades, hsl));
      hipLaunchKernelGGL(k_half_nyquist, dim3((unsigned)blocks), dim3(256), 0, stream, fp, n, K::B, h0, spec,
                         h0_full ? (const float4*)nullptr : h0row, ranks, blk, (const SpectrumConsts*)nullptr);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess || hsl.nstrips < 1)  // a rank past the last strip only builds the Nyquist-row term
        return e;
      // slab items keep fewer pairs in VGPRs: with four, the SLAB store addressing spills 8-16 B (at
      // N = 8192 already with two; one fits)
      constexpr int HKS = LOGN == 13 ? 1 : kHalfHK - 1;
      auto kern = k_cols_half<LOGN, kStream, kStream, true, true, false, 1, 1, K::B, true, false, kHalfHL, HKS>;
      const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + K::LDS1 + kHalfHL * K::WG1 * 16;
      int grid = persistent_grid(kern, K::WG1, lds, fp.cascades * hsl.nstrips, cus);
      if (grid > hs_blocks)
        grid = hs_blocks;
      hipLaunchKernelGGL(kern, dim3(grid), dim3(K::WG1), lds, stream, fp, h0, (float4*)nullptr, (float4*)nullptr,
                         (float2*)nullptr, tw, hs, hsl, (unsigned char*)send, h0_full ? 1 : 0,
                         (const SpectrumConsts*)nullptr);
      return hipGetLastError();
    }
  });
}

// The row pass over row-major fields (strip-dealt slabs after k_half_to_rows, and whole grids of
// 8192/16384 after the four-step column pass). N = 16384 (T = 1024, one row per workgroup): the
// XS x transform (barriers 14 -> 6 per image). tw: this size's table, followed by the N/16-point
// table for the sizes the four-step paths serve (ocean_fft_create appends it for 8192 and 16384).
static int rm_rows_variant = 1;  // tools/microbench A/B (same translation unit): 0 = the plain transform

template <int LOGN>
hipError_t launch_rm_rows(const FrameParams& fp, const float4* rm_ab, const float4* rm_de, const float2* rm_c,
                          const float4* spec, float4* maps, float* jac, const FoamParams& foam, const float2* tw,
                          int rows, int kp, hipStream_t stream, int cus)
{
  using S = FftShape<LOGN>;
  constexpr int RPW = S::T >= 1024 ? 1 : 2;
  if constexpr (RPW == 1)
  {
    if (rm_rows_variant != 0)
    {
      auto kern = k_rows_half<LOGN, kStream, kStream, 0, 1, true, true, 1, 1, 4, 2, true, true>;
      const int lds = XsCfg<LOGN>::LDS;
      const int grid = persistent_grid(kern, S::T, lds, fp.cascades * rows, cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(S::T), lds, stream, fp, rm_ab, rm_de, rm_c, spec, maps, jac, foam, tw,
                         rows, kp, tw + S::TW_ENTRIES);
      return hipGetLastError();
    }
  }
  auto kern = k_rows_half<LOGN, kStream, kStream, 0, RPW, true, true>;
  const int lds = ((S::TW_ENTRIES * 8 + 15) / 16) * 16 + lds_row_slots<LOGN>(RPW) * 8;
  const int grid = persistent_grid(kern, S::T * RPW, lds, fp.cascades * (rows / RPW), cus);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(S::T * RPW), lds, stream, fp, rm_ab, rm_de, rm_c, spec, maps, jac, foam, tw,
                     rows, kp, (const float2*)nullptr);
  return hipGetLastError();
}

hipError_t launch_half_slab_rows(int logn, const FrameParams& fp, const HalfSlab& hsl, const void* recv, float4* rm_ab,
                                 float4* rm_de, float2* rm_c, float4* maps, float* jac, const FoamParams& foam,
                                 const float2* tw, hipStream_t stream, int cus)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (!HalfCfg<LOGN>::SLAB_SUPPORTED)
      return hipErrorInvalidValue;
    else
    {
      using S = FftShape<LOGN>;
      const int n = S::N, B = spectrum_block(LOGN), C = fp.cascades;
      if (hsl.w % kHalfToRowsTY != 0)
        return hipErrorInvalidValue;
      const size_t part = (size_t)C * hsl.S * hsl.w * B, blk = half_slab_block_bytes(LOGN, C, hsl);
      const float4* spec = reinterpret_cast<const float4*>((const unsigned char*)recv +
                                                           half_slab_spec_offset(LOGN, C, hsl));  // block 0's copy
      const int kp = half_strips(LOGN) * B;
      const int tiles = C * ((half_strips(LOGN) + hsl.S - 1) / hsl.S) *
                        ((hsl.S * B + kHalfToRowsTU - 1) / kHalfToRowsTU) * (hsl.w / kHalfToRowsTY);
      const int tgrid = (one_shot_grids(cus) || tiles < cus * 4) ? tiles : cus * 4;
      const unsigned char* in = (const unsigned char*)recv;
      constexpr int KB = ColFirstCfg<LOGN>::B;
      hipLaunchKernelGGL((k_half_to_rows<float4, KB>), dim3(tgrid), dim3(256), 0, stream, C, n, hsl, in, (size_t)0, blk, rm_ab);
      hipLaunchKernelGGL((k_half_to_rows<float4, KB>), dim3(tgrid), dim3(256), 0, stream, C, n, hsl, in, part * 16, blk, rm_de);
      hipLaunchKernelGGL((k_half_to_rows<float2, KB>), dim3(tgrid), dim3(256), 0, stream, C, n, hsl, in, part * 32, blk, rm_c);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess)
        return e;
      return launch_rm_rows<LOGN>(fp, rm_ab, rm_de, rm_c, spec, maps, jac, foam, tw, hsl.w, kp, stream, cus);
      return hipGetLastError();
    }
  });
}

bool ifft_fourstep_supported(int logn) { return logn == 13 || logn == 14; }

size_t ifft_fourstep_work_texels(int logn, int wc) { return ((size_t)1 << logn) * (size_t)wc; }

// Rows in place, then per slab of wc columns: step 1 (images -> work slab), step 2 (slab -> images).
// Bytes: 3 x 32 per texel (the in-place order: 2 x 32, but its column pass reads and writes 16-B
// pieces at N = 16384). Measured (tools/microbench/ifft4bench, profiles/r02_ifft4bench.log), one
// 16384^2 image: in place 7.26 ms, four-step 5.05 ms (wc 2048); at 8192 the in-place order (two
// columns per item, 32-B pieces) stays ahead, 4.78 vs 4.96 ms for 4 images.

hipError_t launch_ifft_fourstep(int logn, int n_images, float4* images, float4* work, int wc, const float2* tw,
                                const float2* tw2, hipStream_t stream, int cus)
{
  if (!ifft_fourstep_supported(logn))
    return hipErrorInvalidValue;
  const int n = 1 << logn;
  if (wc < 64 || wc > n || n % wc != 0 || (wc & 63) != 0)
    return hipErrorInvalidValue;
  hipError_t e = launch_rows_ifft(logn, n_images, images, tw, stream, cus);
  if (e != hipSuccess)
    return e;
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (LOGN < 13)
      return hipErrorInvalidValue;
    else
    {
      constexpr int LOGN2 = LOGN - 4;
      using K2 = ColCfg<LOGN2>;
      auto k1 = k_cols4_step1<LOGN>;
      auto k2 = k_cols4_step2<LOGN2>;
      const int lds2 = lds_bytes_cols<LOGN2>();
      for (int im = 0; im < n_images; im++)
        for (int x0 = 0; x0 < n; x0 += wc)
        {
          float4* img = images + ((size_t)im << (2 * LOGN));
          const int g1 = persistent_grid(k1, 256, 0, (wc / 64) * ((n / 16) / 4), cus);
          hipLaunchKernelGGL(k1, dim3(g1), dim3(256), 0, stream, 1, x0, wc, img, work, tw);
          const int g2 = persistent_grid(k2, K2::WG, lds2, 16 * (wc / K2::C), cus);
          hipLaunchKernelGGL(k2, dim3(g2), dim3(K2::WG), lds2, stream, 1, x0, wc, work, img, tw2);
          const hipError_t le = hipGetLastError();
          if (le != hipSuccess)
            return le;
        }
      return hipSuccess;
    }
  });
}

// ---- whole grids of N = 8192 / 16384 on one rank: four-step column pass (k_gen4_step1/2) ----
bool gen4_supported(int logn) { return logn == 13 || logn == 14; }

int gen4_h0_block() { return kGen4Block; }

size_t gen4_row_texels(int logn, int cascades)
{
  const int n = 1 << logn, kp = n / 2 + spectrum_block(logn);  // Gen4Cfg::KP
  return (size_t)cascades * n * (size_t)((kp + 15) / 16 * 16);
}

size_t gen4_buffer_bytes(int logn, int cascades)
{
  return 40 * gen4_row_texels(logn, cascades) + (size_t)cascades * 2 * ((size_t)1 << logn) * sizeof(float4);
}

hipError_t launch_gen4_columns(int logn, const FrameParams& fp, const float4* h0, void* buf, const float2* tw,
                               hipStream_t stream, int cus)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (LOGN < 13)
      return hipErrorInvalidValue;
    else
    {
      using G = Gen4Cfg<LOGN>;
      constexpr int N = G::N, KP = G::KP;
      // the Nyquist-row term after the three parts
      float4* spec = reinterpret_cast<float4*>((unsigned char*)buf + 40 * gen4_row_texels(LOGN, fp.cascades));
      long blocks = ((long)fp.cascades * N + 255) / 256;
      if (blocks > (long)cus * 4)
        blocks = (long)cus * 4;
      hipLaunchKernelGGL(k_half_nyquist, dim3((unsigned)blocks), dim3(256), 0, stream, fp, N, kGen4Block, h0, spec,
                         (const float4*)nullptr, 1, (size_t)0, (const SpectrumConsts*)nullptr);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess)
        return e;
      auto k1 = k_gen4_step1<LOGN>;
      const int items = fp.cascades * ((KP + 63) / 64) * (N / 16 / 4);
      hipLaunchKernelGGL(k1, dim3(persistent_grid(k1, 256, 0, items, cus)), dim3(256), 0, stream, fp, h0,
                         (unsigned char*)buf, tw);
      return hipGetLastError();
    }
  });
}

hipError_t launch_gen4_rows(int logn, const FrameParams& fp, const void* buf, float4* rm_ab, float4* rm_de, float2* rm_c,
                            float4* maps, float* jac, const FoamParams& foam, const float2* tw, const float2* tw2,
                            hipStream_t stream, int cus)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    if constexpr (LOGN < 13)
      return hipErrorInvalidValue;
    else
    {
      using G = Gen4Cfg<LOGN>;
      constexpr int N = G::N, KP = G::KP, PITCH = G::PITCH, LOGN2 = LOGN - 4;
      // 8 columns per workgroup at N2 = 1024 (512 threads, two per CU: 2.145 -> 2.015 ms for the three
      // parts at 16384, tools/microbench/gen4bench); ColCfg's 16 at N2 = 512 (already 512 threads)
      constexpr int CI = ColCfg<LOGN2>::C * FftShape<LOGN2>::T >= 1024 ? ColCfg<LOGN2>::C / 2 : ColCfg<LOGN2>::C;
      constexpr int WG2 = FftShape<LOGN2>::T * CI;
      const int C = fp.cascades;
      const size_t part = gen4_row_texels(LOGN, C);
      const float4* wab = reinterpret_cast<const float4*>(buf);
      const float4* wde = wab + part;
      const float4* wc = wde + part;  // gc (float2 texels) viewed as pairs of columns
      const float4* spec = reinterpret_cast<const float4*>((const unsigned char*)buf + 40 * part);
      const int lds2 = ((FftShape<LOGN2>::TW_ENTRIES * 8 + 15) / 16) * 16 + CI * FftShape<LOGN2>::PADDED * 8;
      auto sp = k_gen4_step2<LOGN2, true, CI>;
      auto sc = k_gen4_step2<LOGN2, false, CI>;
      const int gp = persistent_grid(sp, WG2, lds2, C * 16 * ((KP + CI - 1) / CI), cus);
      const int gcg = persistent_grid(sc, WG2, lds2, C * 16 * (((KP + 1) / 2 + CI - 1) / CI), cus);
      hipLaunchKernelGGL(sp, dim3(gp), dim3(WG2), lds2, stream, C, KP, PITCH, wab, rm_ab, tw2);
      hipLaunchKernelGGL(sp, dim3(gp), dim3(WG2), lds2, stream, C, KP, PITCH, wde, rm_de, tw2);
      hipLaunchKernelGGL(sc, dim3(gcg), dim3(WG2), lds2, stream, C, (KP + 1) / 2, PITCH / 2, wc,
                         reinterpret_cast<float4*>(rm_c), tw2);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess)
        return e;
      return launch_rm_rows<LOGN>(fp, rm_ab, rm_de, rm_c, spec, maps, jac, foam, tw, N, PITCH, stream, cus);
    }
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

hipError_t launch_rows_ifft_rows(int logn, int rows, float4* data, const float2* tw, hipStream_t stream, int cus)
{
  return with_logn(logn, [&](auto L) -> hipError_t {
    constexpr int LOGN = decltype(L)::value;
    using R = RowCfg<LOGN>;
    auto kern = k_rows_ifft<LOGN>;
    int lds = lds_bytes_rows<LOGN>();
    int items = (rows + R::RPW - 1) / R::RPW;
    int grid = persistent_grid(kern, R::WG, lds, items, cus);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(R::WG), lds, stream, rows, data, tw);
    return hipGetLastError();
  });
}

hipError_t launch_rows_ifft(int logn, int n_images, float4* images, const float2* tw, hipStream_t stream, int cus)
{
  return launch_rows_ifft_rows(logn, n_images << logn, images, tw, stream, cus);
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
