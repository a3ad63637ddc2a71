// ocean_internal.h — types shared between the device code and the C-ABI implementation.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace oceanfft
{

// Waves::GeneratorSettings (src/Generator.h:12-30) == spectrumSettings UBO (spectrum.compute:10-27).
struct OceanSettings
{
  int32_t seed[2];
  float U_10;
  float theta_0;
  float F;
  float g;
  float swell;
  float h;
  float displacement;
  float time;
  float planeSize;
  float scale;
  float spread;
  int32_t boundWavelength;
  float wavelengthMin;
  float wavelengthMax;
};
static_assert(sizeof(OceanSettings) == 64, "GeneratorSettings is 64 bytes");

constexpr int kMaxCascades = 64;  // cascades per launch (kernel-argument tables below)
constexpr int kMaxSurfaceCascades = 16;

// Surface consumer (resources/waveShader.glsl): the maps one cascade binds, plus its planeSize and
// displacement scale (src/Renderer.cpp:62-72).
struct SurfaceCascade
{
  const float4* height;
  const float4* disp;
  const float* jac;
  float plane;
  float scale;
};
struct SurfaceParams
{
  int count;  // cascades
  int n;      // map side (power of two)
  SurfaceCascade c[kMaxSurfaceCascades];
  // null: the stages sample the maps; else the surface atlas [cascade][2][n * n] (launch_surface):
  // (h, Dx, Dz, 0) for the vertex stage, (dh/dx, dh/dz, dDx/dx, dDz/dz) for the normal stage
  float4* atlas;
};
// The reference plane mesh and camera (waveShader.glsl:77-98); res == 0: explicit positions.
struct SurfacePlane
{
  int res;
  float cam_x, cam_y, cam_z, fwd_x, fwd_z;
};

// Per-cascade values the evolve/row kernel needs (passed by value: no per-frame H2D copy).
struct CascadeFrame
{
  float dk;    // 2*pi/planeSize, evaluated in fp32 exactly as spectrum.compute:189
  float time;  // accumulated in fp32 like src/Generator.cpp:50
  float g;
  float h;
};

struct FrameParams
{
  int cascades;
  int pad[3];
  CascadeFrame c[kMaxCascades];
};

struct FoamParams
{
  float displacement[kMaxCascades];
};

// Slab decomposition of one N x N grid over `ranks` GPUs (ranks == 1: the whole grid). This rank
// owns columns [x0, x0 + w) in the column pass and rows [rank*w, rank*w + w) in the row pass,
// w = N / ranks. Pass 1 writes its output in destination-block order (block q = rows q*w..q*w+w-1),
// so one equal-split all-to-all turns it into the row pass's input.
struct SlabGeom
{
  int x0;
  int w;
};

// Half-spectrum strip-dealt layout (slabs of any N >= 1024, and whole grids of N = 8192 / 16384).
// The STRIPS = N / (2B) + 1 kept strips (columns u >= 0, then the Nyquist strip x = 0..B-1) are
// dealt S per rank, rank r taking [r S, min(r S + S, STRIPS)). Pass 1 writes block q (rows
// [q w, q w + w)) of its output as three parts of C * S * w * B elements: gab float4 | gde float4 |
// gc float2, element ((c S + sl) w + yl) B + b; then the frame's Nyquist-row term [c][2][N] float4.
struct HalfSlab
{
  int strip0;   // first global strip of this rank
  int nstrips;  // strips this rank transforms (<= S)
  int S;        // strip slots per block
  int w;        // rows per block = rows of this rank's row pass
};

// Four-step column pass of one rank (N = 8192 / 16384; whole grids: P = 1), SURVEY §8e. The
// N/2 regular kept columns u' (x = N/2 + u') are dealt cols = N / (2P) per rank; rank P - 1 also
// transforms the Nyquist column u = -N/2 (x = 0) as its local column `cols`. Step 1 writes the rank's
// parts [c][N][lp]; step 2 writes its output rows straight into destination-block order: block q
// (rows [q w, q w + w), bound for rank q) = gab | gde | gc parts [c][w][lp] (16, 16, 8 B elements),
// then the frame's Nyquist-row term [c][2][N] float4. After the equal-split all-to-all the row pass
// reads row y's columns from the P source blocks directly (RowSrc): no transpose.
struct Gen4Geom
{
  int u0;            // first regular kept column of this rank
  int cols;          // regular kept columns of this rank, N / (2P) (a multiple of 64)
  int nyq;           // 1: this rank also transforms the Nyquist column (local column `cols`)
  int lp;            // row pitch (texels) of the parts and of the block fields: cols + 16
  int w;             // rows per block, N / P
  int ranks;         // P
  size_t h0_cstride; // h0 texels per cascade
  size_t h0_reg;     // texel offset in a cascade's h0 of the 64-column block holding local column 0
  size_t h0_nyq;     // texel offset of the 64-column block whose first column is x = 0
  size_t blk_bytes;  // exchange block bytes
};

// Row-pass source of row-major fields (k_rows_half RM): element u in [0, N/2) of local row y of
// cascade c sits at ab + (u / cpr) * src_stride + ((c * rows + y) * lp + u % cpr) * 16 (de likewise,
// c with 8-B elements); the Nyquist column u = -N/2 in source block nyq_src at column cpr.
struct RowSrc
{
  const unsigned char* ab;
  const unsigned char* de;
  const unsigned char* c;
  size_t src_stride;  // bytes between source blocks
  int cpr;            // columns per source block (a multiple of 64)
  int lp;             // row pitch in elements
  int nyq_src;        // source block of the Nyquist column
};

// h0 is stored strip-blocked [xb][y][blk]; blk = spectrum_block(log2 N). x0/width select a column
// slab (width <= 0: the whole grid).
int spectrum_block(int logn);
hipError_t launch_generate_spectrum(const OceanSettings& s, int n, float4* h0, hipStream_t stream, int cus, int x0 = 0,
                                    int width = 0, int blk = 0);  // blk 0: spectrum_block(log2 N)
// Half-spectrum generator path (whole grids, N = 1024 .. 4096): pass 1 (+ the Nyquist-row term
// into spec, 2 * cascades rows of N float4) and pass 2. Field buffers: half_field_texels(logn) per
// cascade each for gab, gcd (float4) and ge (float2).
bool half_spectrum_supported(int logn);
size_t half_field_texels(int logn);
// hs (optional): H scratch of half_hs_bytes(logn, hs_blocks) bytes; pass 1 then evolves each texel
// once (grid capped at hs_blocks) instead of once per field round.
size_t half_hs_bytes(int logn, int blocks);  // also the strip-dealt path's
// seed_consts (optional, device array of one seed_consts_bytes() record per cascade, needs hs): the
// fused re-seed frame — pass 1 evaluates h0 itself and neither reads nor writes the h0 image.
// h0's strip width for the whole-grid half path: the half-strip pass (4096, <= 2 cascades) reads
// 2-column h0 strips (k_cols_half HB), the whole-strip pass the 4-column ones (spectrum_block)
int half_h0_block(int logn, int cascades);
// the layout the column pass writes / the row pass reads (launch_common.h HalfFieldLayout)
struct HalfFieldLayout;
HalfFieldLayout half_cols_layout(int logn, int cascades);
HalfFieldLayout half_rows_layout(int logn, int cascades, int variant);
// h0_blk: the strip width h0 is blocked in (0: spectrum_block; 2 only where the pass runs on half
// strips, launch_common.h half_h0_block)
hipError_t launch_half_columns(int logn, const FrameParams& fp, const float4* h0, float4* gab, float4* gcd, float2* ge,
                               float4* spec, const float2* tw, hipStream_t stream, int cus, float2* hs, int hs_blocks,
                               const void* seed_consts = nullptr, int h0_blk = 0);
// generateSpectrum's settings-only constants (host, the oracle's fp32 expressions), as a device record
size_t seed_consts_bytes();
void seed_consts(const OceanSettings& s, int n, void* out);
hipError_t launch_half_rows(int logn, const FrameParams& fp, const float4* gab, const float4* gcd, const float2* ge,
                            const float4* rcorr, float4* maps, float* jac, const FoamParams& foam, const float2* tw,
                            hipStream_t stream, int cus);
// The Nyquist-row term of the half-spectrum paths (k_half_nyquist): spec[c][2][N] from row y = 0 of
// h0 (h0row [c][N] when given, else the whole grid's h0 blocked blk columns wide; seed: evaluated in
// place), written `copies` times copy_stride bytes apart (one copy per exchange block), or with dst
// (the one-sided exchange) copy k at dst[k] + dst_off.
hipError_t launch_half_nyquist(const FrameParams& fp, int n, int blk, const float4* h0, float4* spec, const float4* h0row,
                               int copies, size_t copy_stride, const void* seed, hipStream_t stream, int cus,
                               const uint64_t* dst = nullptr, size_t dst_off = 0);
// One-sided slab exchange (ocean_peers): the frame signals. A wait polls flags[word0 .. word0 + ranks)
// of this rank until each reaches `target`, giving up after deadline_ticks of the device wall clock
// (err[0] then records word0 + 1, and later waits return at once).
struct PeerWait
{
  const uint32_t* flags;
  int word0;
  int ranks;
  uint32_t target;
  long long deadline_ticks;
  uint32_t* err;
};
hipError_t launch_peer_wait(const PeerWait& w, hipStream_t stream);
// Stores `value` into word `word` of every rank's flags (flags[q]: device array of ranks pointers).
hipError_t launch_peer_signal(uint32_t* const* flags, int ranks, int word, uint32_t value, hipStream_t stream);
// The same after writing back every XCD's L2 (the puts' stores); counter: a word of this rank's flags.
hipError_t launch_peer_signal_release(uint32_t* const* flags, int ranks, int word, uint32_t value, uint32_t* counter,
                                      hipStream_t stream);
// Strip-dealt half-spectrum path (HalfSlab): N = 1024 .. 16384. Columns: the Nyquist-row term (from
// h0 when h0_full, i.e. the whole grid's blocked h0, else from h0row = row 0 of every column) into
// every destination block of `send`, and pass 1 of the rank's strips into the blocks (ranks *
// half_slab_block_bytes). Rows: the received blocks -> row-major fields rm_ab / rm_de / rm_c
// (half_slab_row_texels each), then pass 2 over the rank's w rows with block 0's Nyquist-row term.
bool half_slab_supported(int logn);
int half_strips(int logn);
size_t half_slab_block_bytes(int logn, int cascades, const HalfSlab& h);
size_t half_slab_row_texels(int logn, int cascades, int w);
hipError_t launch_generate_spectrum_row(const OceanSettings& s, int n, float4* row, hipStream_t stream);
struct Gen4Put;
// put (the one-sided exchange): blocks and the Nyquist-row term go to put->dst[q] after put->wait;
// the whole pass runs on `stream` (put->stream must be null or equal).
hipError_t launch_half_slab_columns(int logn, const FrameParams& fp, const HalfSlab& hsl, int ranks, const float4* h0,
                                    bool h0_full, const float4* h0row, void* send, const float2* tw,
                                    hipStream_t stream, int cus, float2* hs, int hs_blocks, const Gen4Put* put = nullptr);
hipError_t launch_half_slab_rows(int logn, const FrameParams& fp, const HalfSlab& hsl, const void* recv, float4* rm_ab,
                                 float4* rm_de, float2* rm_c, float4* maps, float* jac, const FoamParams& foam,
                                 const float2* tw, const float2* tw2, hipStream_t stream, int cus);
hipError_t launch_rows_ifft_rows(int logn, int rows, float4* data, const float2* tw, hipStream_t stream, int cus);
// The four-step column pass (Gen4Geom; N = 8192 / 16384, whole grids and slabs of P <= 16). h0: the
// whole grid's image blocked gen4_h0_block() columns wide (whole_h0), or the rank's columns
// (gen4_geom's h0_* offsets). Columns: step 1 into `parts` (gen4_parts_bytes), then the Nyquist-row
// term into every block of `send` and step 2 into the destination blocks of `send` (ranks *
// blk_bytes). One-sided exchange (put != null): no send buffer; block q (term included) goes to
// put->dst[q], a device table of ranks addresses (this rank's block in rank q's receive slot), after
// put->wait (the peers have released the slots), on put->cus CUs (0: cus).
// Rows: the row pass over the w rows of the received blocks. tw2: the N/16-point twiddle table.
bool gen4_supported(int logn);
int gen4_h0_block();
Gen4Geom gen4_geom(int logn, int cascades, int rank, int ranks, bool whole_h0);
size_t gen4_parts_bytes(int logn, int cascades, const Gen4Geom& g);
struct Gen4Put
{
  const uint64_t* dst;
  const PeerWait* wait;          // null: no wait
  int cus;
  hipEvent_t start = nullptr;    // profiling: recorded before the wait and the put kernels
  hipStream_t stream = nullptr;  // the put kernels' stream (null: step 1's), after `handoff`
  hipEvent_t handoff = nullptr;  // recorded on step 1's stream after step 1 when `stream` is set
  void* parts = nullptr;         // the caller's parts slot (null: the generator's)
};
hipError_t launch_gen4_columns(int logn, const FrameParams& fp, const Gen4Geom& g, const float4* h0, const float4* h0row,
                               void* parts, void* send, const float2* tw, const float2* tw2, hipStream_t stream, int cus,
                               const Gen4Put* put = nullptr);
hipError_t launch_gen4_rows(int logn, const FrameParams& fp, const Gen4Geom& g, const void* recv, float4* maps, float* jac,
                            const FoamParams& foam, const float2* tw, const float2* tw2, hipStream_t stream, int cus);
// The N/16-point twiddle table that the four-step paths (gen4, the standalone EncodeIFFT at 8192 /
// 16384) and the XS row pass of 16384 read: ocean_fft_create appends it exactly for these sizes, and
// the launchers that need it fail on a null tw2 instead of reading past the table.
bool fourstep_table(int logn);
// Standalone EncodeIFFT at N = 8192 / 16384: rows in place, then the column transform in four steps
// through a work slab of N x wc texels (ifft_fourstep_work_texels), wc columns at a time. tw2: the
// N/16-point twiddle table.
bool ifft_fourstep_supported(int logn);
size_t ifft_fourstep_work_texels(int logn, int wc);
hipError_t launch_ifft_fourstep(int logn, int n_images, float4* images, float4* work, int wc, const float2* tw,
                                const float2* tw2, hipStream_t stream, int cus);
// Standalone EncodeIFFT, column-first through a work image of n_images * N^2 texels (N = 4096).
bool ifft_colfirst_supported(int logn);
hipError_t launch_ifft_colfirst(int logn, int n_images, float4* images, float4* work, const float2* tw,
                                hipStream_t stream, int cus);
// Standalone EncodeIFFT at N = 8192: the radix-2 pre-stage column pass into a work image of
// n_images * N^2 texels, then the row pass back into the images (16384: kernels for microbench A/B
// only, launch_ifft_pre_t). twn: the N-point twiddle table; twm: the 4096-point table
// (ocean_fft_create appends it for the ifft_pre_supported sizes).
bool ifft_pre_supported(int logn);
hipError_t launch_ifft_pre(int logn, int n_images, float4* images, float4* work, const float2* twn, const float2* twm,
                           hipStream_t stream, int cus);
// p.atlas non-null: the maps are first repacked into it (surface_atlas_texels(p) float4), then sampled
// from it; bit-identical to the direct path.
hipError_t launch_surface(const SurfaceParams& p, const SurfacePlane& plane, const float2* xz, int64_t count,
                          float4* out, hipStream_t stream, int cus);
size_t surface_atlas_texels(const SurfaceParams& p);
bool surface_use_atlas(const SurfaceParams& p, int64_t points);
hipError_t launch_hash(const uint32_t* xy, int count, uint32_t* raw, float2* uv, hipStream_t stream);
hipError_t launch_debug_copy(void* dst, const void* src, size_t bytes, int workgroups, hipStream_t stream);
// Generator frame: pass 1 (evolve + y iFFT, destination-block-ordered output), pass 2 (x iFFT +
// maps + Jacobian). keep: evolved amplitudes kept live between the two packed images (0, 8, 16).
hipError_t launch_cols_evolve(int logn, const FrameParams& fp, const SlabGeom& g, const float4* h0, float4* inter,
                              const float2* tw, hipStream_t stream, int cus, int keep);
int default_keep(int logn);
// Smallest slab width (N / ranks) the column/row pass work items fit in.
int slab_min_width(int logn);
// True when pass 2 needs the B == 1 transpose into a row-major scratch buffer (N = 16384).
bool rows_need_transpose(int logn);
hipError_t launch_rows_final(int logn, int cascades, const SlabGeom& g, const float4* inter, float4* scratch,
                             float4* maps, float* jac, const FoamParams& foam, const float2* tw, hipStream_t stream,
                             int cus);
// EncodeIFFT on row-major images, in place: row pass then column pass.
hipError_t launch_rows_ifft(int logn, int n_images, float4* images, const float2* tw, hipStream_t stream,
                            int cus);
hipError_t launch_cols(int logn, int n_images, float4* images, const float2* tw, hipStream_t stream, int cus);
int twiddle_entries(int logn);

}  // namespace oceanfft
