// ocean_capi.cpp — implementation of the C ABI in include/oceanfft.h.
//
// Host-side orchestration of the reference's FFTCalculator / Generator (src/FFTCalculator.cpp,
// src/Generator.cpp) over the HIP kernels in ocean_kernels.hip. No CPU fallback exists: without a
// GPU every entry point fails with OCEAN_ERR_NO_DEVICE / OCEAN_ERR_HIP.
#include "oceanfft.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "ocean_internal.h"

using namespace oceanfft;

static_assert(sizeof(ocean_settings) == sizeof(OceanSettings), "settings layout");

namespace
{
thread_local std::string g_err;

int fail(int code, const std::string& msg)
{
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what)
{
  return fail(OCEAN_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr, what)                                                                        \
  do                                                                                               \
  {                                                                                                \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess)                                                                          \
      return hip_fail(e_, what);                                                                   \
  } while (0)

int log2_exact(size_t n)
{
  int l = 0;
  while (((size_t)1 << l) < n)
    l++;
  return ((size_t)1 << l) == n ? l : -1;
}

struct EventPair
{
  int kind;
  hipEvent_t a, b;
};
}  // namespace

struct ocean_fft
{
  int n = 0;
  int logn = 0;
  int device = 0;
  int device_cus = 0;  // CUs of the device
  int cus = 0;         // CU budget persistent grids are sized for (ocean_fft_set_cu_budget)
  hipStream_t stream = nullptr;
  float2* twiddles = nullptr;  // two-level table, see FftShape in device/fft.h
  float2* tw2 = nullptr;       // the N/16-point table after it (fourstep_table sizes), else null
  float2* twm = nullptr;       // the 4096-point table after that (ifft_pre_supported sizes), else null
  float4* work = nullptr;      // column-first EncodeIFFT work image (the reference's workImage)
  int work_images = 0;
  size_t work_texels = 0;      // four-step EncodeIFFT (N = 16384): work slab of N x kFourStepSlab texels
  float4* surf_atlas = nullptr;  // the surface consumer's repacked maps (launch_surface), grown on demand
  size_t surf_atlas_texels = 0;
};

// Four-step EncodeIFFT work slab width at N = 16384 (tools/microbench/ifft4bench,
// profiles/r02_ifft4bench.log: 2048 columns 5.05 ms, whole image 5.39, in place 7.26)
constexpr int kFourStepSlab = 2048;

struct ocean_generator
{
  ocean_fft* fft = nullptr;
  int cascades = 0;
  int rank = 0, ranks = 1;  // slab decomposition of one grid (ranks == 1: whole grids, batched)
  SlabGeom geom{};          // this rank's column slab [x0, x0 + w) and row slab width w
  std::vector<ocean_settings> settings;
  bool update_spectrum = true;  // src/Generator.h:72
  float4* h0 = nullptr;         // [cascade][w/B][N][B] strip-blocked column slab (B = spectrum_block)
  float4* inter = nullptr;      // [cascade][ranks][2][w/B][w][B] after the y pass (destination-block order)
  float4* scratch = nullptr;    // [cascade][2][w][N] row-major, only when B == 1 (N = 16384)
  float4* maps = nullptr;       // [cascade][2][w][N]: heightMap, displacementMap rows (row-major)
  float* jac = nullptr;         // [cascade][w][N]
  // half-spectrum path (ranks == 1, N = 1024 .. 4096; ocean_generator_set_half_spectrum)
  bool half = false;
  FrameParams frame{};    // the last column pass's per-cascade values (the row pass needs dk)
  float2* hs = nullptr;    // pass-1 H scratch, half_hs_bytes(logn, device CUs)
  float4* gab = nullptr;  // [cascade][strip][N][4]: y-transformed (H, kz H) for u >= 0 + Nyquist strip
  float4* gcd = nullptr;  // (kz H/|k|, kz^2 H/|k|)
  float2* ge = nullptr;   // H/|k|
  float4* spec = nullptr; // [cascade][2][N]: the Nyquist-row term R
  // half-spectrum paths of slabs (N >= 1024) and of whole grids of N = 8192 / 16384: the four-step
  // column pass (gen4, N = 8192 / 16384, default) or the strip-dealt one (hsl)
  bool hslab = false;
  bool slab = false;  // created by ocean_generator_create_slab (also with ranks == 1)
  HalfSlab hsl{};
  Gen4Geom g4{};
  float4* h0row = nullptr;                            // slabs: [cascade][N], row y = 0 of every column
  float4* rm_ab = nullptr;                            // strip-dealt: row-major fields [cascade][w][kp] after the exchange
  float4* rm_de = nullptr;
  float2* rm_c = nullptr;
  unsigned char* parts = nullptr;                     // four-step: step 1's output [field][cascade][N][lp]
  unsigned char* xbuf = nullptr;                      // internal exchange buffer (ranks == 1, or null send/recv)
  size_t xbuf_bytes = 0;
  // fused re-seed frames (blocked half path): h0 evaluated inside pass 1, the h0 image left stale
  void* seedc = nullptr;                 // device: one seed_consts record per cascade
  std::vector<unsigned char> seedc_host; // what seedc holds
  bool h0_stale = false;                 // the h0 image is not written yet (materialise_h0)
  std::vector<ocean_settings> seed_settings;  // the settings the last fused re-seed evaluated
  // N = 8192 / 16384: the four-step column pass writing destination-block order (launch_gen4_columns
  // / _rows); off: the strip-dealt column pass + transposes. ocean_generator_set_four_step.
  bool four_step = true;
  int h0_block = 0;                          // strip width the h0 image was last written with
  std::vector<ocean_settings> h0_settings;   // the settings it was written from
  // the settings h0 was last seeded from (written or fused): a requested re-seed with the same
  // h0 inputs (every field but `time`) would reproduce h0 bit for bit, so it is skipped
  std::vector<ocean_settings> seeded;
  bool memo_h0 = true;  // ocean_generator_set_h0_memo
  // ocean_generator_slab_frame[_pipelined]: the library's own exchange buffers over RCCL, two slots
  // (frame f in slot f % 2), the exchange on its own stream
  unsigned char* xsend[2] = {nullptr, nullptr};
  unsigned char* xrecv[2] = {nullptr, nullptr};
  size_t xslot_bytes = 0;
  hipStream_t comm_stream = nullptr;
  hipEvent_t cols_done[2] = {nullptr, nullptr}, xchg_done[2] = {nullptr, nullptr}, rows_done[2] = {nullptr, nullptr};
  bool rows_recorded[2] = {false, false};
  int pending_slot = -1;           // slot whose row pass is still to be issued
  FrameParams slot_frame[2]{};     // the column pass's per-cascade values of the frame in each slot
  FoamParams slot_foam[2]{};       // and the settings' displacement its row pass uses
  int64_t frames_issued = 0;
  // the one-sided exchange bound to this generator (ocean_peers_create), and the event that orders its
  // put stream after h0 writes on the generator's stream
  ocean_peers* peers = nullptr;
  hipEvent_t put_h0 = nullptr;
  // Events, not stream handles: the peers' streams (and a caller's) may be destroyed or replaced
  // between frames, and a recorded event stays valid (a stale `cols_stream`).
  // cols_ev: the last strip-dealt / four-step column pass on its own stream (step 1 of a split put
  // frame); the next column pass waits for it, on whatever stream (step 1 rewrites the parts; the
  // strip-dealt pass reuses its H scratch); a no-op when both run on one stream.
  // h0r_ev: the end of that pass's last h0 / h0row reader (the put stream's Nyquist-row kernel, which
  // waited for step 1): every h0 / seed-constant write on the generator's stream waits for it.
  hipEvent_t cols_ev = nullptr, h0r_ev = nullptr;
  bool cols_ev_valid = false;
  // ocean_generator_set_frame_overlap (blocked half path): frame f's column pass on `side` into field
  // slot f % 2, beside frame f - 1's row pass on the generator's stream
  bool overlap = false;
  hipStream_t side = nullptr;
  float4 *gab2 = nullptr, *gcd2 = nullptr, *spec2 = nullptr;
  float2* ge2 = nullptr;
  hipEvent_t ocols[2] = {nullptr, nullptr}, orows[2] = {nullptr, nullptr}, oh0 = nullptr;
  bool orows_valid[2] = {false, false};
  int oslot = 0;
  bool h0_dirty = false;  // h0 (or the fused re-seed constants) written on the generator's stream since the side stream last waited
  bool profiling = false;
  std::vector<EventPair> pending;
  std::vector<hipEvent_t> pool;
  double ms[4] = {0, 0, 0, 0};         // per kind: 0 h0, 1 column pass, 2 row pass, 3 the put inside 1
  int64_t launches[4] = {0, 0, 0, 0};
};

static void peers_detach(ocean_peers* p);  // the one-sided exchange section below
static bool peers_pending(const ocean_peers* p);

extern "C" {

const char* ocean_last_error(void) { return g_err.c_str(); }

const char* ocean_version(void) { return "oceanfft 0.1 (gfx950)"; }

void ocean_default_settings(ocean_settings* s)
{
  // src/Generator.h:14-29
  std::memset(s, 0, sizeof(*s));
  s->seed[0] = 12342;
  s->seed[1] = 8934;
  s->U_10 = 40.0f;
  s->theta_0 = 25.0f;
  s->F = 800000.0f;
  s->g = 9.8f;
  s->swell = 0.5f;
  s->h = 100.0f;
  s->displacement = 0.4f;
  s->time = 0.0f;
  s->planeSize = 40.0f;
  s->scale = 1.0f;
  s->spread = 0.2f;
  s->boundWavelength = 0;
  s->wavelengthMin = 0.0f;
  s->wavelengthMax = 0.0f;
}

int ocean_device_count(void)
{
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess)
    return 0;
  return n;
}

int ocean_fft_create(ocean_fft** out, size_t texture_size, void* hip_stream)
{
  if (!out)
    return fail(OCEAN_ERR_INVALID, "ocean_fft_create: out is null");
  *out = nullptr;
  int logn = log2_exact(texture_size);
  if (logn < 4 || logn > 14)
    return fail(OCEAN_ERR_INVALID, "ocean_fft_create: texture_size must be a power of two in [16, 16384], got " +
                                       std::to_string(texture_size));
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(OCEAN_ERR_NO_DEVICE, "ocean_fft_create: no HIP device visible");

  auto* f = new ocean_fft();
  f->n = (int)texture_size;
  f->logn = logn;
  f->stream = (hipStream_t)hip_stream;
  hipError_t e = hipGetDevice(&f->device);
  if (e == hipSuccess)
    e = hipDeviceGetAttribute(&f->device_cus, hipDeviceAttributeMultiprocessorCount, f->device);
  f->cus = f->device_cus;
  if (e != hipSuccess)
  {
    delete f;
    return hip_fail(e, "ocean_fft_create: device query");
  }

  // Twiddle table exp(+2 pi i e / N), two levels (FFTCalculator's pass table analogue,
  // src/FFTCalculator.cpp:14-32): [0, TB) = low part, [TB, TB+TA) = high part. The four-step
  // EncodeIFFT (N = 16384) appends the N/16-point table.
  std::vector<float2> tab;
  const double two_pi = 6.283185307179586476925286766559;
  auto append_table = [&](int lg) {
    const int lb = lg / 2, tb = 1 << lb, ta = 1 << (lg - lb);
    const double len = (double)(1 << lg);
    for (int e2 = 0; e2 < tb; e2++)
    {
      double a = two_pi * e2 / len;
      tab.push_back(make_float2((float)std::cos(a), (float)std::sin(a)));
    }
    for (int e2 = 0; e2 < ta; e2++)
    {
      double a = two_pi * ((double)e2 * tb) / len;
      tab.push_back(make_float2((float)std::cos(a), (float)std::sin(a)));
    }
  };
  append_table(logn);
  const size_t tw2_at = tab.size();
  if (fourstep_table(logn))
    append_table(logn - 4);
  const size_t twm_at = tab.size();
  if (ifft_pre_supported(logn))
    append_table(12);
  e = hipMalloc(&f->twiddles, tab.size() * sizeof(float2));
  if (e == hipSuccess)
    e = hipMemcpy(f->twiddles, tab.data(), tab.size() * sizeof(float2), hipMemcpyHostToDevice);
  if (e != hipSuccess)
  {
    if (f->twiddles)
      (void)hipFree(f->twiddles);
    delete f;
    return hip_fail(e, "ocean_fft_create: twiddle table");
  }
  if (fourstep_table(logn))
    f->tw2 = f->twiddles + tw2_at;
  if (ifft_pre_supported(logn))
    f->twm = f->twiddles + twm_at;
  *out = f;
  return OCEAN_OK;
}

int ocean_fft_destroy(ocean_fft* fft)
{
  if (!fft)
    return OCEAN_OK;
  if (fft->twiddles)
    (void)hipFree(fft->twiddles);
  if (fft->work)
    (void)hipFree(fft->work);
  if (fft->surf_atlas)
    (void)hipFree(fft->surf_atlas);
  delete fft;
  return OCEAN_OK;
}

size_t ocean_fft_texture_resolution(const ocean_fft* fft) { return fft ? (size_t)fft->n : 0; }

int ocean_fft_device_cus(const ocean_fft* fft) { return fft ? fft->device_cus : 0; }

int ocean_fft_set_cu_budget(ocean_fft* fft, int cus)
{
  if (!fft)
    return fail(OCEAN_ERR_INVALID, "ocean_fft_set_cu_budget: null plan");
  if (cus < 0 || cus > fft->device_cus)
    return fail(OCEAN_ERR_INVALID, "ocean_fft_set_cu_budget: budget outside [0, device CUs]");
  fft->cus = cus == 0 ? fft->device_cus : cus;
  return OCEAN_OK;
}

int ocean_fft_encode_ifft_batch(ocean_fft* fft, float* images, int n_images)
{
  if (!fft || !images || n_images < 1)
    return fail(OCEAN_ERR_INVALID, "ocean_fft_encode_ifft_batch: null plan/image or n_images < 1");
  auto* img = reinterpret_cast<float4*>(images);
  const bool pre = fft->logn == 13 && fft->twm != nullptr;  // 8192: the radix-2 pre-stage column pass
  if (ifft_colfirst_supported(fft->logn) || pre)
  {
    // column-first through a work image of up to 2 GiB (8 images at N = 4096, 2 at 8192)
    const int chunk = std::max(1, (int)(((size_t)2 << 30) / ((size_t)fft->n * fft->n * sizeof(float4))));
    const int want = n_images < chunk ? n_images : chunk;
    if (fft->work_images < want)
    {
      float4* w = nullptr;
      if (hipMalloc(&w, (size_t)want * fft->n * fft->n * sizeof(float4)) == hipSuccess)
      {
        if (fft->work)
          (void)hipFree(fft->work);
        fft->work = w;
        fft->work_images = want;
        fft->work_texels = (size_t)want * fft->n * fft->n;
      }
      else
        (void)hipGetLastError();  // no room for the work image: the in-place passes below
    }
    if (fft->work)
    {
      for (int first = 0; first < n_images; first += fft->work_images)
      {
        const int count = n_images - first < fft->work_images ? n_images - first : fft->work_images;
        float4* first_img = img + (size_t)first * fft->n * fft->n;
        if (pre)
          HIP_TRY(launch_ifft_pre(fft->logn, count, first_img, fft->work, fft->twiddles, fft->twm, fft->stream, fft->cus),
                  "pre-stage EncodeIFFT");
        else
          HIP_TRY(launch_ifft_colfirst(fft->logn, count, first_img, fft->work, fft->twiddles, fft->stream, fft->cus),
                  "column-first EncodeIFFT");
      }
      return OCEAN_OK;
    }
  }
  if (ifft_fourstep_supported(fft->logn) && fft->logn == 14)
  {
    // rows in place, then the column transform in four steps through a work slab of N x 2048
    // texels (512 MiB): every access a >= 256-B row piece instead of one-column 16-B pieces
    const size_t want = ifft_fourstep_work_texels(fft->logn, kFourStepSlab);
    if (fft->work_texels < want)
    {
      float4* w = nullptr;
      if (hipMalloc(&w, want * sizeof(float4)) == hipSuccess)
      {
        if (fft->work)
          (void)hipFree(fft->work);
        fft->work = w;
        fft->work_texels = want;
        fft->work_images = 0;
      }
      else
        (void)hipGetLastError();  // no room for the slab: the in-place passes below
    }
    if (fft->work_texels >= want)
    {
      HIP_TRY(launch_ifft_fourstep(fft->logn, n_images, img, fft->work, kFourStepSlab, fft->twiddles, fft->tw2,
                                   fft->stream, fft->cus),
              "four-step EncodeIFFT");
      return OCEAN_OK;
    }
  }
  HIP_TRY(launch_rows_ifft(fft->logn, n_images, img, fft->twiddles, fft->stream, fft->cus), "row pass");
  HIP_TRY(launch_cols(fft->logn, n_images, img, fft->twiddles, fft->stream, fft->cus), "column pass");
  return OCEAN_OK;
}

int ocean_fft_encode_ifft(ocean_fft* fft, float* image) { return ocean_fft_encode_ifft_batch(fft, image, 1); }

int ocean_fft_synchronize(ocean_fft* fft)
{
  if (!fft)
    return fail(OCEAN_ERR_INVALID, "ocean_fft_synchronize: null plan");
  HIP_TRY(hipStreamSynchronize(fft->stream), "hipStreamSynchronize");
  return OCEAN_OK;
}

}  // extern "C"

namespace
{
hipEvent_t take_event(ocean_generator* g)
{
  if (!g->pool.empty())
  {
    hipEvent_t e = g->pool.back();
    g->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

// Runs `launch` bracketed by events when profiling is on.
template <typename F>
hipError_t timed(ocean_generator* g, int kind, F&& launch, hipStream_t stream = nullptr)
{
  if (!g->profiling)
    return launch();
  if (!stream)
    stream = g->fft->stream;
  EventPair p{kind, take_event(g), take_event(g)};
  hipError_t e = hipEventRecord(p.a, stream);
  if (e != hipSuccess)
    return e;
  e = launch();
  if (e != hipSuccess)
    return e;
  e = hipEventRecord(p.b, stream);
  g->pending.push_back(p);
  return e;
}
}  // namespace

extern "C" {

// ---------------------------------------------------------------------------------------------
// Generator
// ---------------------------------------------------------------------------------------------
static hipError_t half_buffers(ocean_generator* g)
{
  const size_t t = half_field_texels(g->fft->logn) * g->cascades;
  hipError_t e = hipSuccess;
  if (!g->gab)
    e = hipMalloc(&g->gab, t * sizeof(float4));
  if (e == hipSuccess && !g->gcd)
    e = hipMalloc(&g->gcd, t * sizeof(float4));
  if (e == hipSuccess && !g->ge)
    e = hipMalloc(&g->ge, t * sizeof(float2));
  if (e == hipSuccess && !g->spec)
    e = hipMalloc(&g->spec, (size_t)g->cascades * 2 * g->fft->n * sizeof(float4));
  if (e == hipSuccess && !g->hs)  // pass 1's H scratch: one slice per resident block (1 per CU)
    e = hipMalloc(&g->hs, half_hs_bytes(g->fft->logn, g->fft->device_cus));
  return e;
}

// The strip-dealt path's geometry: STRIPS kept strips dealt S = ceil(STRIPS / ranks) per rank.
static HalfSlab half_slab_geom(int logn, int rank, int ranks)
{
  const int strips = half_strips(logn);
  HalfSlab h{};
  h.S = (strips + ranks - 1) / ranks;
  h.strip0 = rank * h.S;
  h.nstrips = std::max(0, std::min(h.S, strips - h.strip0));
  h.w = (1 << logn) / ranks;
  return h;
}

static bool uses_gen4(const ocean_generator* g)
{
  return g->four_step && g->hslab && gen4_supported(g->fft->logn);
}

// strip width of the h0 image the current frame path reads (the whole-grid half path at <= 2
// cascades of 4096: 2-column strips, one per half-strip item, launch_common.h half_h0_block)
static int h0_block(const ocean_generator* g)
{
  if (uses_gen4(g))
    return gen4_h0_block();
  if (g->half && g->ranks == 1)
    return half_h0_block(g->fft->logn, g->cascades);
  return spectrum_block(g->fft->logn);
}

// h0 texels per cascade: the whole grid (ranks == 1), or the largest of a slab's layouts (its column
// slab, its dealt strips, its four-step columns blocked 64 wide), so switching paths needs no reallocation
static size_t h0_texels(const ocean_generator* g)
{
  const size_t full = (size_t)g->fft->n * g->geom.w;  // the full path's column slab (whole grid: N^2)
  if (g->ranks == 1)
    return full;
  const size_t strips = (size_t)g->hsl.nstrips * spectrum_block(g->fft->logn) * g->fft->n;
  size_t t = std::max(full, strips);
  if (gen4_supported(g->fft->logn))
    t = std::max(t, g->g4.h0_cstride);
  return t;
}

static size_t hslab_xbuf_bytes(const ocean_generator* g)
{
  if (uses_gen4(g))
    return (size_t)g->ranks * g->g4.blk_bytes;
  return (size_t)g->ranks * half_slab_block_bytes(g->fft->logn, g->cascades, g->hsl);
}

// The buffers of the current half-spectrum slab path (allocated when the path is first used; a path
// switch keeps the other path's buffers). Four-step: step 1's parts and the exchange blocks (ranks ==
// 1: one block, read back by the row pass). Strip-dealt: the row-major fields and the H scratch.
static hipError_t hslab_buffers(ocean_generator* g)
{
  const int logn = g->fft->logn, C = g->cascades;
  hipError_t e = hipSuccess;
  if (uses_gen4(g))
  {
    if (!g->parts)
      e = hipMalloc(&g->parts, gen4_parts_bytes(logn, C, g->g4));
  }
  else
  {
    const size_t rt = half_slab_row_texels(logn, C, g->hsl.w);
    if (!g->rm_ab)
      e = hipMalloc(&g->rm_ab, rt * sizeof(float4));
    if (e == hipSuccess && !g->rm_de)
      e = hipMalloc(&g->rm_de, rt * sizeof(float4));
    if (e == hipSuccess && !g->rm_c)
      e = hipMalloc(&g->rm_c, rt * sizeof(float2));
    if (e == hipSuccess && !g->hs)
      e = hipMalloc(&g->hs, half_hs_bytes(logn, g->fft->device_cus));
  }
  const size_t xb = hslab_xbuf_bytes(g);
  if (e == hipSuccess && g->xbuf_bytes < xb)
  {
    if (g->xbuf)
      (void)hipFree(g->xbuf);
    g->xbuf = nullptr;
    g->xbuf_bytes = 0;
    e = hipMalloc(&g->xbuf, xb);
    if (e == hipSuccess)
      g->xbuf_bytes = xb;
  }
  if (e == hipSuccess && g->ranks > 1 && !g->h0row)
    e = hipMalloc(&g->h0row, (size_t)C * g->fft->n * sizeof(float4));
  return e;
}

static hipError_t full_buffers(ocean_generator* g)
{
  const size_t slab = (size_t)g->fft->n * g->geom.w * g->cascades;
  hipError_t e = hipSuccess;
  if (!g->inter)
    e = hipMalloc(&g->inter, slab * 2 * sizeof(float4));
  if (e == hipSuccess && rows_need_transpose(g->fft->logn) && !g->scratch)
    e = hipMalloc(&g->scratch, slab * 2 * sizeof(float4));
  return e;
}

static int generator_alloc(ocean_generator** out, ocean_fft* fft, int cascades, int rank, int ranks, bool is_slab)
{
  auto* g = new ocean_generator();
  g->fft = fft;
  g->cascades = cascades;
  g->rank = rank;
  g->ranks = ranks;
  g->geom.w = fft->n / ranks;
  g->geom.x0 = rank * g->geom.w;
  g->settings.resize(cascades);
  for (auto& s : g->settings)
    ocean_default_settings(&s);
  const size_t slab = (size_t)fft->n * g->geom.w;  // texels per cascade image slab
  g->half = ranks == 1 && half_spectrum_supported(fft->logn);
  // slabs of N >= 1024 and whole grids above the blocked half path's sizes: strip-dealt half spectrum
  g->slab = is_slab;
  g->half = g->half && !is_slab;
  g->hslab = !g->half && half_slab_supported(fft->logn) && (is_slab || fft->logn > 12);
  g->hsl = half_slab_geom(fft->logn, rank, ranks);
  if (gen4_supported(fft->logn))
  {
    g->g4 = gen4_geom(fft->logn, cascades, rank, ranks, ranks == 1);
    // one h0 cascade stride for every writer and reader (generate_spectrum_with, k_gen4,
    // ocean_generator_initial_spectrum): the largest of the layouts, as allocated
    g->g4.h0_cstride = h0_texels(g);
  }
  // the strip-dealt column pass reads cascade c's strips at (c * nstrips + s) * N * B, which equals
  // h0_texels(g) * c only for one cascade: slabs are single-grid (ocean_generator_create_slab)
  if (is_slab && cascades != 1)
  {
    delete g;
    return fail(OCEAN_ERR_INVALID, "generator allocation: a slab generator holds exactly one cascade");
  }
  hipError_t e = hipMalloc(&g->h0, h0_texels(g) * cascades * sizeof(float4));
  if (e == hipSuccess && !g->half && !g->hslab)
    e = full_buffers(g);
  if (e == hipSuccess && g->half)
    e = half_buffers(g);
  if (e == hipSuccess && g->hslab)
    e = hslab_buffers(g);
  if (e == hipSuccess)
    e = hipMalloc(&g->maps, slab * cascades * 2 * sizeof(float4));
  if (e == hipSuccess)
    e = hipMalloc(&g->jac, slab * cascades * sizeof(float));
  // Textures start zeroed like the reference's (Data = nullptr) images.
  if (e == hipSuccess)
    e = hipMemsetAsync(g->h0, 0, h0_texels(g) * cascades * sizeof(float4), fft->stream);
  if (e == hipSuccess)
    e = hipMemsetAsync(g->maps, 0, slab * cascades * 2 * sizeof(float4), fft->stream);
  if (e == hipSuccess)
    e = hipMemsetAsync(g->jac, 0, slab * cascades * sizeof(float), fft->stream);
  if (e != hipSuccess)
  {
    int code = (e == hipErrorOutOfMemory) ? OCEAN_ERR_OOM : OCEAN_ERR_HIP;
    ocean_generator_destroy(g);
    return fail(code, std::string("generator allocation: ") + hipGetErrorString(e));
  }
  *out = g;
  return OCEAN_OK;
}

int ocean_generator_create(ocean_generator** out, ocean_fft* fft, int cascades)
{
  if (!out || !fft)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_create: null argument");
  *out = nullptr;
  if (cascades < 1 || cascades > OCEAN_MAX_CASCADES)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_create: cascades must be in [1, 64]");
  return generator_alloc(out, fft, cascades, 0, 1, false);
}

int ocean_generator_create_slab(ocean_generator** out, ocean_fft* fft, int rank, int ranks)
{
  if (!out || !fft)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_create_slab: null argument");
  *out = nullptr;
  const int blk = spectrum_block(fft->logn);
  if (ranks < 1 || ranks > 16 || (ranks & (ranks - 1)) != 0 || rank < 0 || rank >= ranks)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_create_slab: ranks must be a power of two in [1, 16], 0 <= rank < ranks");
  const int w = fft->n / ranks;
  if (w % blk != 0 || w < fft->n / 16 || w < slab_min_width(fft->logn))
    return fail(OCEAN_ERR_INVALID, "ocean_generator_create_slab: N / ranks = " + std::to_string(w) +
                                       " is below this size's minimum slab width " +
                                       std::to_string(slab_min_width(fft->logn)));
  return generator_alloc(out, fft, 1, rank, ranks, true);
}

int ocean_generator_destroy(ocean_generator* g)
{
  if (!g)
    return OCEAN_OK;
  // A pipelined slab frame still in flight: its exchange may be running on comm_stream (the
  // communicator must outlive the generator, include/oceanfft.h). Drain it before the slots go.
  if (g->comm_stream)
    (void)hipStreamSynchronize(g->comm_stream);
  if (g->peers)
    peers_detach(g->peers);
  if (g->fft)
    (void)hipStreamSynchronize(g->fft->stream);
  for (auto& p : g->pending)
  {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  for (auto ev : g->pool)
    (void)hipEventDestroy(ev);
  if (g->h0)
    (void)hipFree(g->h0);
  if (g->inter)
    (void)hipFree(g->inter);
  if (g->scratch)
    (void)hipFree(g->scratch);
  if (g->maps)
    (void)hipFree(g->maps);
  if (g->jac)
    (void)hipFree(g->jac);
  for (int k = 0; k < 2; k++)
  {
    for (hipEvent_t ev : {g->cols_done[k], g->xchg_done[k], g->rows_done[k]})
      if (ev)
        (void)hipEventDestroy(ev);
    for (void* p : {(void*)g->xsend[k], (void*)g->xrecv[k]})
      if (p)
        (void)hipFree(p);
  }
  if (g->comm_stream)
    (void)hipStreamDestroy(g->comm_stream);
  if (g->put_h0)
    (void)hipEventDestroy(g->put_h0);
  for (hipEvent_t ev : {g->cols_ev, g->h0r_ev})
    if (ev)
      (void)hipEventDestroy(ev);
  if (g->side)
  {
    (void)hipStreamSynchronize(g->side);
    (void)hipStreamDestroy(g->side);
  }
  for (hipEvent_t ev : {g->ocols[0], g->ocols[1], g->orows[0], g->orows[1], g->oh0})
    if (ev)
      (void)hipEventDestroy(ev);
  for (void* p : {(void*)g->gab2, (void*)g->gcd2, (void*)g->ge2, (void*)g->spec2})
    if (p)
      (void)hipFree(p);
  for (void* p : {(void*)g->gab, (void*)g->gcd, (void*)g->ge, (void*)g->spec, (void*)g->hs, (void*)g->h0row, g->seedc,
                  (void*)g->rm_ab, (void*)g->rm_de, (void*)g->rm_c, (void*)g->parts, (void*)g->xbuf})
    if (p)
      (void)hipFree(p);
  delete g;
  return OCEAN_OK;
}

int ocean_generator_cascades(const ocean_generator* g) { return g ? g->cascades : 0; }

ocean_settings* ocean_generator_settings(ocean_generator* g, int c)
{
  if (!g || c < 0 || c >= g->cascades)
  {
    fail(OCEAN_ERR_INVALID, "ocean_generator_settings: cascade out of range");
    return nullptr;
  }
  return &g->settings[c];
}


// h0, h0row and the fused re-seed constants are written on the generator's stream; a column pass that
// ran on another stream (the one-sided exchange's step-1 / put streams) may still be reading them
static int wait_h0_readers(ocean_generator* g)
{
  if (g->cols_ev_valid)
    HIP_TRY(hipStreamWaitEvent(g->fft->stream, g->h0r_ev, 0), "h0 write: wait for the last column pass");
  return OCEAN_OK;
}

// generateSpectrum with the given per-cascade settings (the current ones, or those a fused re-seed
// frame evaluated h0 with, when that h0 image is materialised later)
static int generate_spectrum_with(ocean_generator* g, const std::vector<ocean_settings>& settings)
{
  {
    const int rc = wait_h0_readers(g);  // write-after-read on h0 (a pipelined put frame still in flight)
    if (rc != OCEAN_OK)
      return rc;
  }
  g->h0_dirty = true;
  g->h0_stale = false;
  g->h0_block = h0_block(g);
  g->h0_settings = settings;
  g->seeded = settings;
  ocean_fft* f = g->fft;
  const size_t slab = h0_texels(g);
  for (int c = 0; c < g->cascades; c++)
  {
    OceanSettings s;
    std::memcpy(&s, &settings[c], sizeof(s));
    if (uses_gen4(g) && g->ranks > 1)
    {
      // this rank's kept columns x = N/2 + u0 .. (blocked 64 wide), rank P - 1 also the block of
      // x = 0 .. 63 (the Nyquist column x = 0 is its first); plus row 0 of every column
      const Gen4Geom& q = g->g4;
      float4* base = g->h0 + q.h0_cstride * c;
      HIP_TRY(timed(g, 0, [&] {
                hipError_t e = launch_generate_spectrum(s, f->n, base + q.h0_reg, f->stream, f->cus,
                                                        f->n / 2 + q.u0, q.cols, gen4_h0_block());
                if (e == hipSuccess && q.nyq)
                  e = launch_generate_spectrum(s, f->n, base + q.h0_nyq, f->stream, f->cus, 0, gen4_h0_block(),
                                               gen4_h0_block());
                if (e == hipSuccess)
                  e = launch_generate_spectrum_row(s, f->n, g->h0row + (size_t)c * f->n, f->stream);
                return e;
              }),
              "generateSpectrum");
      continue;
    }
    if (g->hslab && g->ranks > 1)
    {
      // this rank's strips: the regular ones are columns N/2 + strip*B .. (contiguous), the last
      // global strip is the Nyquist strip x = 0..B-1; plus row 0 of every column (Nyquist-row term)
      const int B = spectrum_block(f->logn), strips = half_strips(f->logn);
      const HalfSlab& h = g->hsl;
      const int nreg = std::max(0, std::min(h.nstrips, strips - 1 - h.strip0));
      float4* base = g->h0 + h0_texels(g) * c;
      HIP_TRY(timed(g, 0, [&] {
                hipError_t e = hipSuccess;
                if (nreg > 0)
                  e = launch_generate_spectrum(s, f->n, base, f->stream, f->cus, f->n / 2 + h.strip0 * B, nreg * B);
                if (e == hipSuccess && nreg < h.nstrips)
                  e = launch_generate_spectrum(s, f->n, base + (size_t)nreg * f->n * B, f->stream, f->cus, 0, B);
                if (e == hipSuccess)
                  e = launch_generate_spectrum_row(s, f->n, g->h0row + (size_t)c * f->n, f->stream);
                return e;
              }),
              "generateSpectrum");
      continue;
    }
    HIP_TRY(timed(g, 0, [&] {
              return launch_generate_spectrum(s, f->n, g->h0 + slab * c, f->stream, f->cus, g->geom.x0, g->geom.w,
                                              g->h0_block);
            }),
            "generateSpectrum");
  }
  return OCEAN_OK;
}

int ocean_generator_generate_spectrum(ocean_generator* g)
{
  if (!g)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_generate_spectrum: null generator");
  return generate_spectrum_with(g, g->settings);
}

// After fused re-seed frames: write the h0 image those frames evaluated (their settings snapshot).
static int materialise_h0(ocean_generator* g)
{
  return g->h0_stale ? generate_spectrum_with(g, g->seed_settings) : OCEAN_OK;
}

// First half of CalculateOcean: time += dt (src/Generator.cpp:50), h0 if requested (:55-59),
// prepareFFT fused with the y direction of both EncodeIFFTs (:63-72). Output in destination-block
// order into `out` (the internal buffer when null).
// True when h0 seeded from `a` and from `b` is the same image: every field but the accumulated
// time (generateSpectrum does not read it, spectrum.compute:157-172).
static bool same_h0_inputs(const std::vector<ocean_settings>& a, const std::vector<ocean_settings>& b)
{
  if (a.size() != b.size())
    return false;
  for (size_t i = 0; i < a.size(); i++)
  {
    ocean_settings x = a[i], y = b[i];
    x.time = y.time = 0.0f;
    if (std::memcmp(&x, &y, sizeof(x)) != 0)
      return false;
  }
  return true;
}

// put (four-step slabs, the one-sided exchange): step 2 stores into the peers' receive slots, on
// col_stream (null: the generator's stream), which first waits for the h0 writes issued so far.
static int generator_columns(ocean_generator* g, float timestep, int update_spectrum, float4* out,
                             const Gen4Put* put = nullptr, hipStream_t col_stream = nullptr)
{
  ocean_fft* f = g->fft;
  for (auto& s : g->settings)
    s.time += timestep;
  const void* seed = nullptr;
  // The reference app asks for a re-seed on every frame (src/Waves.cpp:91-94); when the h0 inputs
  // are unchanged since the last seeding the result would be bit-identical, so it is skipped.
  if (update_spectrum && !g->update_spectrum && g->memo_h0 && same_h0_inputs(g->settings, g->seeded))
    update_spectrum = 0;
  if (g->update_spectrum || update_spectrum)
  {
    // The generator's first seeding writes the h0 image. Explicit re-seeds (the reference app's
    // every-frame CalculateOcean(dt, true)) are fused into pass 1 on the blocked half path; the
    // inlined ocml functions round the same amplitude within an ulp of the seeding kernels' (frames
    // agree to ~1e-7 of max, test_fused_reseed_frames), so the first frame keeps the kernels that
    // slabs and batches are compared with bit-exactly.
    const bool fused = update_spectrum && !g->update_spectrum && g->half && g->hs;
    g->update_spectrum = false;
    if (fused)
    {
      // fused re-seed (src/Generator.cpp:55-59 followed by :63-72): pass 1 evaluates h0 itself
      std::vector<unsigned char> host((size_t)g->cascades * seed_consts_bytes());
      for (int c = 0; c < g->cascades; c++)
      {
        OceanSettings os;
        std::memcpy(&os, &g->settings[c], sizeof(os));
        seed_consts(os, f->n, host.data() + (size_t)c * seed_consts_bytes());
      }
      if (!g->seedc)
        HIP_TRY(hipMalloc(&g->seedc, (size_t)kMaxCascades * seed_consts_bytes()), "seed constants");
      if (host != g->seedc_host)  // pageable source: staged before the call returns
      {
        const int rc = wait_h0_readers(g);
        if (rc != OCEAN_OK)
          return rc;
        HIP_TRY(hipMemcpyAsync(g->seedc, host.data(), host.size(), hipMemcpyHostToDevice, f->stream), "seed constants");
        g->seedc_host.swap(host);
      }
      seed = g->seedc;
      g->h0_dirty = true;
      g->h0_stale = true;
      g->seed_settings = g->settings;
      g->seeded = g->settings;
    }
    else
    {
      int rc = ocean_generator_generate_spectrum(g);
      if (rc != OCEAN_OK)
        return rc;
    }
  }
  else
  {
    int rc = materialise_h0(g);  // the next frames read the h0 image
    if (rc != OCEAN_OK)
      return rc;
    if (g->h0_block != h0_block(g))  // the frame path changed (four-step on/off): same h0, new layout
    {
      rc = generate_spectrum_with(g, g->h0_settings);
      if (rc != OCEAN_OK)
        return rc;
    }
  }
  FrameParams fp{};
  fp.cascades = g->cascades;
  for (int c = 0; c < g->cascades; c++)
  {
    const ocean_settings& s = g->settings[c];
    // spectrum.compute:189 — `2.0 * M_PI / planeSize` in fp32
    fp.c[c].dk = 2.0f * 3.14159265358f / s.planeSize;
    fp.c[c].time = s.time;
    fp.c[c].g = s.g;
    fp.c[c].h = s.h;
  }
  if (g->hslab)
  {
    hipError_t e = hslab_buffers(g);  // the current path's buffers (a path switch allocates here)
    if (e != hipSuccess)
      return fail(e == hipErrorOutOfMemory ? OCEAN_ERR_OOM : OCEAN_ERR_HIP,
                  std::string("column pass buffers: ") + hipGetErrorString(e));
  }
  if (uses_gen4(g) || g->hslab)
  {
    // the column pass's stream (the put or step-1 stream of pipelined one-sided frames) runs after the
    // last column pass on another stream (step 1 rewrites the parts its step 2 read; the strip-dealt
    // pass reuses its H scratch) and after h0 writes
    hipStream_t cs = col_stream ? col_stream : f->stream;
    // both orderings, independently: after the last column pass (whatever stream it ran on), and after
    // the h0 writes on the generator's stream when this pass runs elsewhere
    if (g->cols_ev_valid)
      HIP_TRY(hipStreamWaitEvent(cs, g->cols_ev, 0), "column pass: after the last column pass");
    if (cs != f->stream && g->h0_dirty)
    {
      if (!g->put_h0)
        HIP_TRY(hipEventCreateWithFlags(&g->put_h0, hipEventDisableTiming), "column pass: event");
      HIP_TRY(hipEventRecord(g->put_h0, f->stream), "column pass: stream event");
      HIP_TRY(hipStreamWaitEvent(cs, g->put_h0, 0), "column pass: stream order");
      g->h0_dirty = false;  // only once the wait is enqueued
    }
    // profiling a put: kind 3 brackets the wait + put kernels inside the column pass (kind 1)
    Gen4Put timed_put = put ? *put : Gen4Put{};
    EventPair pp{3, nullptr, nullptr};
    if (put && g->profiling)
    {
      pp.a = take_event(g);
      pp.b = take_event(g);
      timed_put.start = pp.a;
    }
    if (uses_gen4(g))
      HIP_TRY(timed(g, 1, [&] {
                return launch_gen4_columns(f->logn, fp, g->g4, g->h0, g->ranks > 1 ? g->h0row : nullptr,
                                           put && put->parts ? put->parts : g->parts, out ? (void*)out : (void*)g->xbuf,
                                           f->twiddles, f->tw2, cs, f->cus, put ? &timed_put : nullptr);
              }, cs),
              "column pass (half spectrum, four-step)");
    else
      HIP_TRY(timed(g, 1, [&] {
                return launch_half_slab_columns(f->logn, fp, g->hsl, g->ranks, g->h0, g->ranks == 1, g->h0row,
                                                out ? (void*)out : (void*)g->xbuf, f->twiddles, cs, f->cus, g->hs,
                                                f->device_cus, put ? &timed_put : nullptr);
              }, cs),
              "column pass (half spectrum, strip-dealt)");
    if (pp.a)
    {
      HIP_TRY(hipEventRecord(pp.b, put && put->stream ? put->stream : cs), "column pass: put event");
      g->pending.push_back(pp);
    }
    for (hipEvent_t* ev : {&g->cols_ev, &g->h0r_ev})
      if (!*ev)
        HIP_TRY(hipEventCreateWithFlags(ev, hipEventDisableTiming), "column pass: event");
    HIP_TRY(hipEventRecord(g->cols_ev, cs), "column pass: end event");
    // the h0 readers end on the put stream when step 2 runs there (it waited for step 1's handoff)
    HIP_TRY(hipEventRecord(g->h0r_ev, put && put->stream ? put->stream : cs), "column pass: end event");
    g->cols_ev_valid = true;
  }
  else if (put)
    return fail(OCEAN_ERR_INVALID, "column pass: the one-sided exchange needs a half-spectrum slab path (N >= 1024)");
  else if (g->half && g->overlap)
  {
    // frame overlap: this column pass on the side stream into field slot oslot, after the row pass
    // that last read the slot, and after any h0 / seed-constant writes on the generator's stream
    const int s = g->oslot;
    if (g->h0_dirty)
    {
      HIP_TRY(hipEventRecord(g->oh0, f->stream), "overlap: h0 event");
      HIP_TRY(hipStreamWaitEvent(g->side, g->oh0, 0), "overlap: h0 wait");
      g->h0_dirty = false;
    }
    if (g->orows_valid[s])
      HIP_TRY(hipStreamWaitEvent(g->side, g->orows[s], 0), "overlap: slot wait");
    HIP_TRY(timed(g, 1, [&] {
              return launch_half_columns(f->logn, fp, g->h0, s ? g->gab2 : g->gab, s ? g->gcd2 : g->gcd,
                                         s ? g->ge2 : g->ge, s ? g->spec2 : g->spec, f->twiddles, g->side, f->cus,
                                         g->hs, f->device_cus, seed, g->h0_block);
            }, g->side),
            "column pass (half spectrum, overlapped)");
    HIP_TRY(hipEventRecord(g->ocols[s], g->side), "overlap: column event");
  }
  else if (g->half)
    HIP_TRY(timed(g, 1, [&] {
              return launch_half_columns(f->logn, fp, g->h0, g->gab, g->gcd, g->ge, g->spec, f->twiddles, f->stream,
                                         f->cus, g->hs, f->device_cus, seed, g->h0_block);
            }),
            "column pass (half spectrum)");
  else
    HIP_TRY(timed(g, 1, [&] {
              return launch_cols_evolve(f->logn, fp, g->geom, g->h0, out, f->twiddles, f->stream, f->cus,
                                        default_keep(f->logn));
            }),
            "column pass");
  g->frame = fp;
  return OCEAN_OK;
}

static FoamParams current_foam(const ocean_generator* g)
{
  FoamParams foam{};
  for (int c = 0; c < g->cascades; c++)
    foam.displacement[c] = g->settings[c].displacement;
  return foam;
}

// Second half: the x direction of both EncodeIFFTs + computeFoam (src/Generator.cpp:71-80). `frame_foam`:
// the displacement of a pipelined slab frame's own settings (null: the current settings).
// row_stream (half-spectrum slab paths; null: the generator's stream): the pipelined one-sided frame's rows.
// row_cus (> 0): the CUs the row stream may use (a CU-masked stream), which sizes resident grids.
static int generator_rows(ocean_generator* g, const float4* in, const FoamParams* frame_foam = nullptr,
                          hipStream_t row_stream = nullptr, int row_cus = 0)
{
  ocean_fft* f = g->fft;
  const int rcus = row_cus > 0 && row_cus < f->cus ? row_cus : f->cus;
  const FoamParams foam = frame_foam ? *frame_foam : current_foam(g);
  if (uses_gen4(g))
  {
    hipStream_t rs = row_stream ? row_stream : f->stream;
    HIP_TRY(timed(g, 2, [&] {
              return launch_gen4_rows(f->logn, g->frame, g->g4, in ? (const void*)in : (const void*)g->xbuf, g->maps,
                                      g->jac, foam, f->twiddles, f->tw2, rs, rcus);
            }, rs),
            "row pass (half spectrum, four-step)");
  }
  else if (g->hslab)
  {
    hipStream_t rs = row_stream ? row_stream : f->stream;
    HIP_TRY(timed(g, 2, [&] {
              return launch_half_slab_rows(f->logn, g->frame, g->hsl, in ? (const void*)in : (const void*)g->xbuf,
                                           g->rm_ab, g->rm_de, g->rm_c, g->maps, g->jac, foam, f->twiddles,
                                           f->tw2, rs, rcus);
            }, rs),
            "row pass (half spectrum, strip-dealt)");
  }
  else if (row_stream)
    return fail(OCEAN_ERR_INVALID, "row pass: a row stream needs a half-spectrum slab path");
  else if (g->half && g->overlap)
  {
    const int s = g->oslot;
    HIP_TRY(hipStreamWaitEvent(f->stream, g->ocols[s], 0), "overlap: column wait");
    HIP_TRY(timed(g, 2, [&] {
              return launch_half_rows(f->logn, g->frame, s ? g->gab2 : g->gab, s ? g->gcd2 : g->gcd,
                                      s ? g->ge2 : g->ge, s ? g->spec2 : g->spec, g->maps, g->jac, foam, f->twiddles,
                                      f->stream, f->cus);
            }),
            "row pass (half spectrum, overlapped)");
    HIP_TRY(hipEventRecord(g->orows[s], f->stream), "overlap: row event");
    g->orows_valid[s] = true;
    g->oslot = s ^ 1;
  }
  else if (g->half)
    HIP_TRY(timed(g, 2, [&] {
              return launch_half_rows(f->logn, g->frame, g->gab, g->gcd, g->ge, g->spec, g->maps, g->jac, foam,
                                      f->twiddles, f->stream, f->cus);
            }),
            "row pass (half spectrum)");
  else
    HIP_TRY(timed(g, 2, [&] {
              return launch_rows_final(f->logn, g->cascades, g->geom, in, g->scratch, g->maps, g->jac, foam,
                                       f->twiddles, f->stream, f->cus);
            }),
            "row pass");
  return OCEAN_OK;
}

int ocean_generator_set_half_spectrum(ocean_generator* g, int enable)
{
  if (!g)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_set_half_spectrum: null generator");
  if (peers_pending(g->peers))
  {
    const int rc = ocean_peers_flush(g->peers);  // a pipelined one-sided frame in flight lands first
    if (rc != OCEAN_OK)
      return rc;
  }
  if (g->pending_slot >= 0)
  {
    // a pipelined slab frame's column pass wrote its blocks in the current path's layout: its row
    // pass runs before the switch
    const int rc = ocean_generator_slab_flush(g);
    if (rc != OCEAN_OK)
      return rc;
  }
  if (!enable && g->overlap)
  {
    const int rc = ocean_generator_set_frame_overlap(g, 0);
    if (rc != OCEAN_OK)
      return rc;
  }
  const int logn = g->fft->logn;
  const bool blocked = !g->slab && half_spectrum_supported(logn);
  const bool dealt = !blocked && half_slab_supported(logn) && (g->slab || logn > 12);
  if (enable && !blocked && !dealt)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_set_half_spectrum: N = 1024 .. 16384 only");
  const bool was_half = g->half, was_hslab = g->hslab;
  g->half = enable && blocked;
  g->hslab = enable && dealt;
  hipError_t e = hipSuccess;
  if (!enable)
    e = full_buffers(g);
  else if (blocked)
    e = half_buffers(g);
  else
    e = hslab_buffers(g);
  if (e != hipSuccess)
  {
    g->half = was_half;
    g->hslab = was_hslab;
    return fail(e == hipErrorOutOfMemory ? OCEAN_ERR_OOM : OCEAN_ERR_HIP,
                std::string("ocean_generator_set_half_spectrum: ") + hipGetErrorString(e));
  }
  if ((was_hslab && g->ranks > 1) != (g->hslab && g->ranks > 1))
    g->update_spectrum = true;  // a slab's h0 layout changes (its strips or columns <-> its column slab)
  return OCEAN_OK;
}

int ocean_generator_set_frame_overlap(ocean_generator* g, int enable)
{
  if (!g)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_set_frame_overlap: null generator");
  if (enable && !g->half)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_set_frame_overlap: whole grids of N = 1024 .. 4096 on the "
                                   "half-spectrum path only");
  ocean_fft* f = g->fft;
  if (enable && !g->overlap)
  {
    const size_t t = half_field_texels(f->logn) * g->cascades;
    hipError_t e = hipSuccess;
    if (!g->side)
      e = hipStreamCreateWithFlags(&g->side, hipStreamNonBlocking);
    for (hipEvent_t* ev : {&g->ocols[0], &g->ocols[1], &g->orows[0], &g->orows[1], &g->oh0})
      if (e == hipSuccess && !*ev)
        e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    if (e == hipSuccess && !g->gab2)
      e = hipMalloc(&g->gab2, t * sizeof(float4));
    if (e == hipSuccess && !g->gcd2)
      e = hipMalloc(&g->gcd2, t * sizeof(float4));
    if (e == hipSuccess && !g->ge2)
      e = hipMalloc(&g->ge2, t * sizeof(float2));
    if (e == hipSuccess && !g->spec2)
      e = hipMalloc(&g->spec2, (size_t)g->cascades * 2 * f->n * sizeof(float4));
    // the side stream starts after everything issued so far (the last column pass used slot 0 and hs)
    if (e == hipSuccess)
      e = hipEventRecord(g->oh0, f->stream);
    if (e == hipSuccess)
      e = hipStreamWaitEvent(g->side, g->oh0, 0);
    if (e != hipSuccess)
      return fail(e == hipErrorOutOfMemory ? OCEAN_ERR_OOM : OCEAN_ERR_HIP,
                  std::string("ocean_generator_set_frame_overlap: ") + hipGetErrorString(e));
    g->orows_valid[0] = g->orows_valid[1] = false;
    g->oslot = 0;
    g->h0_dirty = false;
    g->overlap = true;
  }
  else if (!enable && g->overlap)
  {
    // later frames run on the generator's stream in slot 0: after every overlapped pass
    for (int s = 0; s < 2; s++)
      if (g->orows_valid[s])
        HIP_TRY(hipStreamWaitEvent(f->stream, g->orows[s], 0), "ocean_generator_set_frame_overlap");
    HIP_TRY(hipEventRecord(g->oh0, g->side), "ocean_generator_set_frame_overlap");
    HIP_TRY(hipStreamWaitEvent(f->stream, g->oh0, 0), "ocean_generator_set_frame_overlap");
    g->overlap = false;
  }
  return OCEAN_OK;
}

int ocean_generator_set_h0_memo(ocean_generator* g, int enable)
{
  if (!g)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_set_h0_memo: null generator");
  g->memo_h0 = enable != 0;
  return OCEAN_OK;
}

int ocean_generator_set_four_step(ocean_generator* g, int enable)
{
  if (!g)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_set_four_step: null generator");
  if (peers_pending(g->peers))
  {
    const int rc = ocean_peers_flush(g->peers);  // a pipelined one-sided frame in flight lands first
    if (rc != OCEAN_OK)
      return rc;
  }
  if (g->pending_slot >= 0)
  {
    const int rc = ocean_generator_slab_flush(g);  // as in ocean_generator_set_half_spectrum
    if (rc != OCEAN_OK)
      return rc;
  }
  g->four_step = enable != 0;  // h0 is re-laid out by the next frame if its strip width changes
  if (g->hslab)
  {
    const hipError_t e = hslab_buffers(g);  // exchange_bytes reports the new path's size from here on
    if (e != hipSuccess)
      return fail(e == hipErrorOutOfMemory ? OCEAN_ERR_OOM : OCEAN_ERR_HIP,
                  std::string("ocean_generator_set_four_step: ") + hipGetErrorString(e));
  }
  return OCEAN_OK;
}

int ocean_generator_frame_bytes(const ocean_generator* g, double per_point[2])
{
  if (!g || !per_point)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_frame_bytes: null argument");
  if (uses_gen4(g))
  {
    // the kept columns u' in [0, N/2) and the Nyquist column: step 1 reads h0 (16) and writes 5
    // complex fields (40), step 2 reads and writes them (40 + 40, into the exchange blocks) | the row
    // pass reads them (40) and writes the maps + Jacobian (36)
    const double n = g->fft->n, kept = (n / 2 + 1) / n;
    per_point[0] = (16.0 + 40.0 + 80.0) * kept;
    per_point[1] = 40.0 * kept + 36.0;
  }
  else if (g->half || g->hslab)
  {
    // h0 of the kept columns (half + the Nyquist strip) + 5 complex fields out; 5 fields in, maps +
    // Jacobian; the strip-dealt path also moves the received fields to row-major (40 in + 40 out)
    const double n = g->fft->n, kept = (n / 2 + spectrum_block(g->fft->logn)) / n;
    per_point[0] = 16.0 * kept + 40.0 * kept;
    per_point[1] = 40.0 * kept + 36.0 + (g->hslab ? 80.0 * kept : 0.0);
  }
  else
  {
    per_point[0] = 48.0;
    per_point[1] = 68.0 + (rows_need_transpose(g->fft->logn) ? 64.0 : 0.0);  // B = 1: the tiled transpose
  }
  return OCEAN_OK;
}

int ocean_generator_calculate(ocean_generator* g, float timestep, int update_spectrum)
{
  if (!g)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_calculate: null generator");
  if (g->ranks != 1)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_calculate: slab generators step with "
                                   "ocean_generator_slab_columns / exchange / ocean_generator_slab_rows");
  float4* buf = g->hslab ? nullptr : g->inter;  // null: the strip-dealt path's own exchange buffer
  int rc = generator_columns(g, timestep, update_spectrum, buf);
  return rc != OCEAN_OK ? rc : generator_rows(g, buf);
}

size_t ocean_generator_exchange_bytes(const ocean_generator* g)
{
  if (!g)
    return 0;
  if (g->hslab)
    return hslab_xbuf_bytes(g);
  return (size_t)g->cascades * 2 * g->fft->n * g->geom.w * sizeof(float4);
}

int ocean_generator_slab_columns(ocean_generator* g, float timestep, int update_spectrum, float* send)
{
  if (!g)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_slab_columns: null generator");
  return generator_columns(g, timestep, update_spectrum,
                           send ? reinterpret_cast<float4*>(send) : (g->hslab ? nullptr : g->inter));
}

int ocean_generator_slab_rows(ocean_generator* g, const float* recv)
{
  if (!g)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_slab_rows: null generator");
  return generator_rows(g, recv ? reinterpret_cast<const float4*>(recv) : (g->hslab ? nullptr : g->inter));
}

// ---------------------------------------------------------------------------------------------
// Slab exchange over RCCL: the equal-split all-to-all between the column and the row pass (SURVEY
// §8e), as P grouped ncclSend / ncclRecv pairs of exchange_bytes / P on the generator's streams.
// ---------------------------------------------------------------------------------------------
}  // extern "C"

struct ocean_comm
{
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0;
  bool owned = false;
};

namespace
{
int nccl_fail(ncclResult_t r, const char* what)
{
  return fail(OCEAN_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}

// The equal-split all-to-all of blk bytes per rank pair, enqueued on `stream`: one group of
// ncclSend / ncclRecv pairs, each block in pieces of at most kExchangePiece bytes (RCCL 2.26 corrupted
// a single send / receive above 1 GiB in a world-size-1 self exchange: tools/rccl_selfcheck.py,
// profiles/r03_rccl_selfcheck.log; a whole 8192^2 block is 1.35 GB).
constexpr size_t kExchangePiece = (size_t)512 << 20;

int exchange_bytes_all_to_all(ocean_comm* c, const unsigned char* send, unsigned char* recv, size_t blk,
                              hipStream_t stream)
{
  ncclResult_t r = ncclGroupStart();
  for (int q = 0; q < c->nranks && r == ncclSuccess; q++)
    for (size_t o = 0; o < blk && r == ncclSuccess; o += kExchangePiece)
    {
      const size_t len = std::min(kExchangePiece, blk - o);
      r = ncclSend(send + q * blk + o, len, ncclUint8, q, c->comm, stream);
      if (r == ncclSuccess)
        r = ncclRecv(recv + q * blk + o, len, ncclUint8, q, c->comm, stream);
    }
  const ncclResult_t e = ncclGroupEnd();
  if (r != ncclSuccess)
    return nccl_fail(r, "slab exchange (ncclSend / ncclRecv)");
  if (e != ncclSuccess)
    return nccl_fail(e, "slab exchange (ncclGroupEnd)");
  return OCEAN_OK;
}

// Enqueue this frame's all-to-all (send slot -> recv slot) on `stream`.
int exchange_blocks(ocean_generator* g, ocean_comm* c, const unsigned char* send, unsigned char* recv,
                    hipStream_t stream)
{
  return exchange_bytes_all_to_all(c, send, recv, ocean_generator_exchange_bytes(g) / g->ranks, stream);
}

// The two exchange slots, the comm stream and its events (first use, or after a path switch that
// changed exchange_bytes).
int frame_slots(ocean_generator* g)
{
  const size_t bytes = ocean_generator_exchange_bytes(g);
  if (g->xslot_bytes < bytes)
  {
    if (g->pending_slot >= 0)
      return fail(OCEAN_ERR_INVALID, "slab frame: the exchange size changed with a frame in flight (flush first)");
    for (int k = 0; k < 2; k++)
      for (unsigned char** p : {&g->xsend[k], &g->xrecv[k]})
      {
        if (*p)
          (void)hipFree(*p);
        *p = nullptr;
      }
    g->xslot_bytes = 0;
    for (int k = 0; k < 2; k++)
    {
      HIP_TRY(hipMalloc(&g->xsend[k], bytes), "slab frame: exchange buffers");
      HIP_TRY(hipMalloc(&g->xrecv[k], bytes), "slab frame: exchange buffers");
    }
    g->xslot_bytes = bytes;
  }
  if (!g->comm_stream)
  {
    HIP_TRY(hipStreamCreateWithFlags(&g->comm_stream, hipStreamNonBlocking), "slab frame: comm stream");
    for (int k = 0; k < 2; k++)
      for (hipEvent_t* ev : {&g->cols_done[k], &g->xchg_done[k], &g->rows_done[k]})
        HIP_TRY(hipEventCreateWithFlags(ev, hipEventDisableTiming), "slab frame: events");
  }
  return OCEAN_OK;
}

int check_comm(const ocean_generator* g, const ocean_comm* c, const char* who)
{
  if (!g || !c || !c->comm)
    return fail(OCEAN_ERR_INVALID, std::string(who) + ": null generator or communicator");
  if (c->nranks != g->ranks || c->rank != g->rank)
    return fail(OCEAN_ERR_INVALID, std::string(who) + ": communicator rank " + std::to_string(c->rank) + " of " +
                                       std::to_string(c->nranks) + " does not match slab rank " +
                                       std::to_string(g->rank) + " of " + std::to_string(g->ranks));
  return OCEAN_OK;
}

// Row pass of the frame in slot s (its own column-pass values: pipelined rows run after the next
// frame's column pass).
int slot_rows(ocean_generator* g, int s)
{
  ocean_fft* f = g->fft;
  HIP_TRY(hipStreamWaitEvent(f->stream, g->xchg_done[s], 0), "slab frame: wait for the exchange");
  const FrameParams newest = g->frame;
  g->frame = g->slot_frame[s];
  const int rc = generator_rows(g, reinterpret_cast<const float4*>(g->xrecv[s]), &g->slot_foam[s]);
  g->frame = newest;
  if (rc != OCEAN_OK)
    return rc;
  HIP_TRY(hipEventRecord(g->rows_done[s], f->stream), "slab frame: events");
  g->rows_recorded[s] = true;
  return OCEAN_OK;
}

// Column pass of frame f into slot f % 2 and its exchange on the comm stream.
int slot_columns_and_exchange(ocean_generator* g, ocean_comm* c, float timestep, int update_spectrum, int& slot)
{
  ocean_fft* f = g->fft;
  const int s = (int)(g->frames_issued % 2);
  int rc = generator_columns(g, timestep, update_spectrum, reinterpret_cast<float4*>(g->xsend[s]));
  if (rc != OCEAN_OK)
    return rc;
  g->slot_frame[s] = g->frame;
  g->slot_foam[s] = current_foam(g);
  HIP_TRY(hipEventRecord(g->cols_done[s], f->stream), "slab frame: events");
  HIP_TRY(hipStreamWaitEvent(g->comm_stream, g->cols_done[s], 0), "slab frame: stream order");
  if (g->rows_recorded[s])  // frame f - 2's row pass has finished reading recv[s]
    HIP_TRY(hipStreamWaitEvent(g->comm_stream, g->rows_done[s], 0), "slab frame: stream order");
  rc = exchange_blocks(g, c, g->xsend[s], g->xrecv[s], g->comm_stream);
  if (rc != OCEAN_OK)
    return rc;
  HIP_TRY(hipEventRecord(g->xchg_done[s], g->comm_stream), "slab frame: events");
  g->frames_issued++;
  slot = s;
  return OCEAN_OK;
}
}  // namespace

extern "C" {

int ocean_comm_unique_id(unsigned char id[OCEAN_COMM_ID_BYTES])
{
  static_assert(OCEAN_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "RCCL unique id size");
  if (!id)
    return fail(OCEAN_ERR_INVALID, "ocean_comm_unique_id: null id");
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess)
    return nccl_fail(r, "ncclGetUniqueId");
  std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return OCEAN_OK;
}

int ocean_comm_create(ocean_comm** out, const unsigned char id[OCEAN_COMM_ID_BYTES], int nranks, int rank)
{
  if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(OCEAN_ERR_INVALID, "ocean_comm_create: null argument or rank outside [0, nranks)");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(OCEAN_ERR_NO_DEVICE, "ocean_comm_create: no HIP device visible");
  ncclUniqueId u;
  std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  auto* c = new ocean_comm();
  const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess)
  {
    delete c;
    return nccl_fail(r, "ncclCommInitRank");
  }
  c->nranks = nranks;
  c->rank = rank;
  c->owned = true;
  *out = c;
  return OCEAN_OK;
}

int ocean_comm_wrap(ocean_comm** out, void* nccl_comm, int nranks, int rank)
{
  if (!out || !nccl_comm || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(OCEAN_ERR_INVALID, "ocean_comm_wrap: null argument or rank outside [0, nranks)");
  *out = nullptr;
  // the exchange addresses peers by these values: they must be the communicator's own
  const ncclComm_t nc = static_cast<ncclComm_t>(nccl_comm);
  int count = 0, user_rank = 0;
  ncclResult_t r = ncclCommCount(nc, &count);
  if (r == ncclSuccess)
    r = ncclCommUserRank(nc, &user_rank);
  if (r != ncclSuccess)
    return nccl_fail(r, "ocean_comm_wrap: ncclCommCount / ncclCommUserRank");
  if (count != nranks || user_rank != rank)
    return fail(OCEAN_ERR_INVALID, "ocean_comm_wrap: the communicator is rank " + std::to_string(user_rank) + " of " +
                                       std::to_string(count) + ", not rank " + std::to_string(rank) + " of " +
                                       std::to_string(nranks));
  auto* c = new ocean_comm();
  c->comm = nc;
  c->nranks = nranks;
  c->rank = rank;
  *out = c;
  return OCEAN_OK;
}

int ocean_comm_destroy(ocean_comm* comm)
{
  if (!comm)
    return OCEAN_OK;
  ncclResult_t r = ncclSuccess;
  if (comm->owned && comm->comm)
    r = ncclCommDestroy(comm->comm);
  delete comm;
  return r == ncclSuccess ? OCEAN_OK : nccl_fail(r, "ncclCommDestroy");
}

int ocean_comm_all_to_all(ocean_comm* comm, const void* send, void* recv, size_t bytes, void* hip_stream)
{
  if (!comm || !comm->comm || (bytes > 0 && (!send || !recv)) || bytes % comm->nranks != 0)
    return fail(OCEAN_ERR_INVALID, "ocean_comm_all_to_all: null argument or bytes not a multiple of the rank count");
  return exchange_bytes_all_to_all(comm, static_cast<const unsigned char*>(send), static_cast<unsigned char*>(recv),
                                   bytes / comm->nranks, (hipStream_t)hip_stream);
}

int ocean_generator_slab_frame(ocean_generator* g, ocean_comm* comm, float timestep, int update_spectrum)
{
  int rc = check_comm(g, comm, "ocean_generator_slab_frame");
  if (rc == OCEAN_OK && g->pending_slot >= 0)
    rc = ocean_generator_slab_flush(g);  // a pipelined frame in flight lands first
  if (rc == OCEAN_OK)
    rc = frame_slots(g);
  int s = 0;
  if (rc == OCEAN_OK)
    rc = slot_columns_and_exchange(g, comm, timestep, update_spectrum, s);
  return rc != OCEAN_OK ? rc : slot_rows(g, s);
}

int ocean_generator_slab_frame_pipelined(ocean_generator* g, ocean_comm* comm, float timestep, int update_spectrum)
{
  int rc = check_comm(g, comm, "ocean_generator_slab_frame_pipelined");
  if (rc == OCEAN_OK)
    rc = frame_slots(g);
  int s = 0;
  if (rc == OCEAN_OK)
    rc = slot_columns_and_exchange(g, comm, timestep, update_spectrum, s);
  if (rc != OCEAN_OK)
    return rc;
  if (g->pending_slot >= 0)
  {
    rc = slot_rows(g, g->pending_slot);
    if (rc != OCEAN_OK)
      return rc;
  }
  g->pending_slot = s;
  return OCEAN_OK;
}

int ocean_generator_slab_flush(ocean_generator* g)
{
  if (!g)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_slab_flush: null generator");
  if (g->pending_slot < 0)
    return OCEAN_OK;
  const int s = g->pending_slot;
  g->pending_slot = -1;
  return slot_rows(g, s);
}

// ---------------------------------------------------------------------------------------------
// The one-sided slab exchange (ocean_peers): the four-step column pass stores block q into rank q's
// receive slot through a peer mapping, and per-frame flag words replace the all-to-all (SURVEY §8e;
// DESIGN.md §6 "one-sided exchange").
// ---------------------------------------------------------------------------------------------
}  // extern "C"

namespace
{
constexpr int kMaxRanks = 16;
constexpr int kReadyWord = 0, kFreedWord = 16, kReleaseCounter = 40, kErrWord = 48, kFlagWords = 64;
constexpr uint32_t kPeerMagic = 0x4f505231;  // "OPR1"

struct PeerHandle
{
  uint32_t magic;
  int32_t rank, ranks;
  uint32_t flags_uncached;
  uint64_t slot_bytes;
  hipIpcMemHandle_t data, flags;
};
static_assert(sizeof(PeerHandle) <= OCEAN_PEER_HANDLE_BYTES, "peer handle size");
}  // namespace

struct ocean_peers
{
  ocean_generator* g = nullptr;
  int rank = 0, ranks = 1;
  size_t blk = 0, slot = 0;        // block bytes, slot bytes (ranks * blk = the exchange bytes)
  unsigned char* data = nullptr;   // this rank's two receive slots
  uint32_t* flags = nullptr;       // this rank's flag words: ready[16] | freed[16] | .. | release counter @ 40 | err @ 48
  bool flags_uncached = false;
  unsigned char* peer_data[kMaxRanks] = {};
  uint32_t* peer_flags[kMaxRanks] = {};
  bool mapped[2 * kMaxRanks] = {};  // data / flags opened with hipIpcOpenMemHandle (closed on destroy)
  bool connected = false;
  uint64_t* table = nullptr;       // device: put destinations [2 slots][16], then the flag arrays [16]
  // pipelined frames: step 1 on s1_stream into parts slot f % 2, the put on put_stream, the row pass
  // on the generator's stream (ocean_peers_set_streams can replace the first two)
  hipStream_t s1_stream = nullptr, put_stream = nullptr, row_stream = nullptr;
  hipStream_t own_s1 = nullptr, own_put = nullptr, own_rows = nullptr;
  int put_cus_per_xcd = 0;           // own streams CU-masked: the put on this many CUs of every XCD
  int row_cus = 0;                   // the CUs the own row stream may use when masked (0: all)
  int caller_row_cus = 0;            // ocean_peers_set_row_cus: the caller's row stream's CUs (0: all)
  hipEvent_t rows_done = nullptr;    // pipelined rows on row_stream -> the generator's stream
  hipEvent_t gen_ready = nullptr;    // the generator's stream -> pipelined rows (caller work on the maps)
  bool failed = false;               // a wait timed out (ocean_peers_synchronize): frames are refused
  unsigned char* parts2 = nullptr;   // step 1's second parts slot
  hipEvent_t s1_done[2] = {nullptr, nullptr}, put_done[2] = {nullptr, nullptr};
  bool put_done_valid[2] = {false, false};
  long long deadline = 0;          // wall-clock ticks
  int timeout_ms = 20000;
  int put_cus = 0;
  int64_t frames = 0;              // frames whose column pass was issued
  int64_t rows = 0;                // frames whose row pass was issued
  FrameParams slot_frame[2]{};
  FoamParams slot_foam[2]{};
};

namespace
{
int peers_deadline(ocean_peers* p)
{
  int khz = 0;
  HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, p->g ? p->g->fft->device : 0),
          "ocean_peers: wall clock rate");
  p->deadline = (long long)(khz > 0 ? khz : 100000) * p->timeout_ms;
  return OCEAN_OK;
}

int check_peers(const ocean_generator* g, const ocean_peers* p, const char* who)
{
  if (!g || !p || p->g != g)
    return fail(OCEAN_ERR_INVALID, std::string(who) + ": null generator, or peers created for another generator");
  if (!p->connected)
    return fail(OCEAN_ERR_INVALID, std::string(who) + ": ocean_peers_connect has not run");
  if (p->failed)
    return fail(OCEAN_ERR_TIMEOUT, std::string(who) + ": a one-sided wait timed out earlier (ocean_peers_synchronize "
                                                      "reported it); the ranks' flags are out of step: destroy and "
                                                      "recreate the peers");
  if (!g->hslab || hslab_xbuf_bytes(g) != p->slot)
    return fail(OCEAN_ERR_INVALID, std::string(who) + ": the generator left the half-spectrum slab path (or its "
                                                      "exchange size changed) since ocean_peers_create");
  return OCEAN_OK;
}

// the device table: dst[s][q] = rank q's slot s + this rank's block offset, then the flag arrays
int peers_table(ocean_peers* p)
{
  uint64_t host[3 * kMaxRanks] = {};
  for (int s = 0; s < 2; s++)
    for (int q = 0; q < p->ranks; q++)
      host[s * kMaxRanks + q] = (uint64_t)(uintptr_t)(p->peer_data[q] + s * p->slot + (size_t)p->rank * p->blk);
  for (int q = 0; q < p->ranks; q++)
    host[2 * kMaxRanks + q] = (uint64_t)(uintptr_t)p->peer_flags[q];
  HIP_TRY(hipMemcpy(p->table, host, sizeof(host), hipMemcpyHostToDevice), "ocean_peers: destination table");
  p->connected = true;
  return OCEAN_OK;
}

PeerWait peer_wait(ocean_peers* p, int word0, int64_t target)
{
  return PeerWait{p->flags, word0, p->ranks, (uint32_t)target, p->deadline, p->flags + kErrWord};
}

uint32_t* const* flag_table(const ocean_peers* p)
{
  return reinterpret_cast<uint32_t* const*>(p->table + 2 * kMaxRanks);
}

// Column pass of frame f = p->frames into every rank's slot f % 2, then this rank's "ready" word (f + 1)
// in every rank's flags. The put waits until every rank has finished reading that slot (frame f - 2's
// row pass). Serial: all on the generator's stream. Pipelined: step 1 on s1_stream into parts slot f % 2
// (after the put of frame f - 2 read that slot), the put on put_stream after step 1, so step 1 of frame
// f + 1 and the row pass of frame f - 1 run beside the put of frame f.
int put_columns(ocean_generator* g, ocean_peers* p, float timestep, int update_spectrum, bool pipelined)
{
  ocean_fft* fs = g->fft;
  const int64_t f = p->frames;
  const int s = (int)(f % 2);
  const PeerWait w = peer_wait(p, kFreedWord, f - 1);
  Gen4Put put{p->table + s * kMaxRanks, f >= 2 ? &w : nullptr, p->put_cus};
  hipStream_t cs = nullptr;
  if (pipelined && uses_gen4(g))
  {
    if (!p->parts2)
      HIP_TRY(hipMalloc(&p->parts2, gen4_parts_bytes(fs->logn, g->cascades, g->g4)), "one-sided exchange: parts slot");
    cs = p->s1_stream;
    put.parts = s ? p->parts2 : g->parts;
    put.stream = p->put_stream;
    put.handoff = p->s1_done[s];
    if (p->put_done_valid[s])
      HIP_TRY(hipStreamWaitEvent(cs, p->put_done[s], 0), "one-sided exchange: parts slot reuse");
  }
  else if (pipelined)
    cs = p->put_stream;  // the strip-dealt pass stores its blocks itself: all of it on the put stream
  else
    for (int k = 0; k < 2; k++)  // a serial frame after pipelined ones: its step 1 rewrites parts slot 0
      if (p->put_done_valid[k])
      {
        HIP_TRY(hipStreamWaitEvent(fs->stream, p->put_done[k], 0), "one-sided exchange: stream order");
        p->put_done_valid[k] = false;
      }
  int rc = generator_columns(g, timestep, update_spectrum, nullptr, &put, cs);
  if (rc != OCEAN_OK)
    return rc;
  hipStream_t ps = pipelined ? p->put_stream : fs->stream;
  HIP_TRY(launch_peer_signal_release(flag_table(p), p->ranks, kReadyWord + p->rank, (uint32_t)(f + 1),
                                     p->flags + kReleaseCounter, ps),
          "one-sided exchange: ready signal");
  if (pipelined)
  {
    HIP_TRY(hipEventRecord(p->put_done[s], ps), "one-sided exchange: events");
    p->put_done_valid[s] = true;
  }
  p->slot_frame[s] = g->frame;
  p->slot_foam[s] = current_foam(g);
  p->frames = f + 1;
  return OCEAN_OK;
}

// Row pass of the oldest frame whose rows are not issued yet: wait for every rank's blocks, rows, then
// this rank's "freed" word (f + 1) in every rank's flags. Serial: on the generator's stream. Pipelined:
// on the peers' row stream, which the generator's stream then waits for (the maps stay ordered on it).
int put_rows(ocean_generator* g, ocean_peers* p, bool pipelined = false)
{
  ocean_fft* f = g->fft;
  const int64_t fr = p->rows;
  if (fr >= p->frames)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_slab_put_rows: no column pass issued for this frame");
  const int s = (int)(fr % 2);
  hipStream_t rs = pipelined ? p->row_stream : f->stream;
  if (rs != f->stream)
  {
    // the row pass rewrites g->maps / jac: after the caller's work on the generator's stream (the
    // header keeps the maps ordered there)
    HIP_TRY(hipEventRecord(p->gen_ready, f->stream), "one-sided exchange: events");
    HIP_TRY(hipStreamWaitEvent(rs, p->gen_ready, 0), "one-sided exchange: stream order");
  }
  HIP_TRY(launch_peer_wait(peer_wait(p, kReadyWord, fr + 1), rs), "one-sided exchange: ready wait");
  const FrameParams newest = g->frame;
  g->frame = p->slot_frame[s];
  const int rc = generator_rows(g, reinterpret_cast<const float4*>(p->data + s * p->slot), &p->slot_foam[s], rs,
                                rs == p->own_rows ? p->row_cus : p->caller_row_cus);
  g->frame = newest;
  if (rc != OCEAN_OK)
    return rc;
  HIP_TRY(launch_peer_signal(flag_table(p), p->ranks, kFreedWord + p->rank, (uint32_t)(fr + 1), rs),
          "one-sided exchange: freed signal");
  if (rs != f->stream)
  {
    HIP_TRY(hipEventRecord(p->rows_done, rs), "one-sided exchange: events");
    HIP_TRY(hipStreamWaitEvent(f->stream, p->rows_done, 0), "one-sided exchange: stream order");
  }
  p->rows = fr + 1;
  return OCEAN_OK;
}

// (Re)create the peers' own streams; with put_cus_per_xcd > 0 CU-masked: the put stream on that many
// CUs of every XCD, the step-1 and row streams on the others. A hipExtStreamCreateWithCUMask bit c is
// CU c / 8 of XCD c % 8, and an XCD whose bits are all clear runs on all its CUs (workgroups are dealt
// to every XCD whatever the mask; tools/xcdmask, profiles/r05_xcdprobe.log): a mask can only split
// each XCD, so the put takes the same share of each.
int peers_streams(ocean_peers* p)
{
  for (hipStream_t* st : {&p->own_s1, &p->own_put, &p->own_rows})
    if (*st)
    {
      HIP_TRY(hipStreamSynchronize(*st), "ocean_peers: streams");
      HIP_TRY(hipStreamDestroy(*st), "ocean_peers: streams");
      *st = nullptr;
    }
  const int cus = p->g->fft->device_cus;
  if (p->put_cus_per_xcd > 0 && cus % 8 == 0 && p->put_cus_per_xcd < cus / 8)
  {
    std::vector<uint32_t> put((cus + 31) / 32, 0u), rest((cus + 31) / 32, 0u);
    for (int c = 0; c < cus; c++)
      (c / 8 < p->put_cus_per_xcd ? put : rest)[c / 32] |= 1u << (c % 32);
    HIP_TRY(hipExtStreamCreateWithCUMask(&p->own_put, (uint32_t)put.size(), put.data()), "ocean_peers: put stream");
    HIP_TRY(hipExtStreamCreateWithCUMask(&p->own_s1, (uint32_t)rest.size(), rest.data()), "ocean_peers: column stream");
    HIP_TRY(hipExtStreamCreateWithCUMask(&p->own_rows, (uint32_t)rest.size(), rest.data()), "ocean_peers: row stream");
    p->row_cus = cus - 8 * p->put_cus_per_xcd;  // resident row-pass grids sized to the masked stream
  }
  else
  {
    for (hipStream_t* st : {&p->own_s1, &p->own_put, &p->own_rows})
      HIP_TRY(hipStreamCreateWithFlags(st, hipStreamNonBlocking), "ocean_peers: streams");
    p->row_cus = 0;
  }
  p->s1_stream = p->own_s1;
  p->put_stream = p->own_put;
  p->row_stream = p->own_rows;
  p->put_done_valid[0] = p->put_done_valid[1] = false;
  return OCEAN_OK;
}

void peers_release(ocean_peers* p)
{
  for (hipStream_t st : {p->s1_stream, p->put_stream, p->row_stream})
    if (st)
      (void)hipStreamSynchronize(st);
  if (p->g && p->g->fft)
    (void)hipStreamSynchronize(p->g->fft->stream);
  for (int q = 0; q < kMaxRanks; q++)
  {
    if (p->mapped[q] && p->peer_data[q])
      (void)hipIpcCloseMemHandle(p->peer_data[q]);
    if (p->mapped[kMaxRanks + q] && p->peer_flags[q])
      (void)hipIpcCloseMemHandle(p->peer_flags[q]);
    p->mapped[q] = p->mapped[kMaxRanks + q] = false;
  }
}
}  // namespace

// a column pass whose row pass is not issued yet (a pipelined frame in flight)
static bool peers_pending(const ocean_peers* p) { return p && p->rows < p->frames; }

// called by ocean_generator_destroy: a generator destroyed before its peers leaves them unusable
static void peers_detach(ocean_peers* p)
{
  if (!p)
    return;
  for (hipStream_t st : {p->s1_stream, p->put_stream, p->row_stream})
    if (st)
      (void)hipStreamSynchronize(st);
  p->g = nullptr;
  p->connected = false;
}

extern "C" {

int ocean_peers_create(ocean_peers** out, ocean_generator* g)
{
  if (!out || !g)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_create: null argument");
  *out = nullptr;
  if (!g->slab || !g->hslab)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_create: a slab generator on a half-spectrum path (N >= 1024)");
  if (g->peers)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_create: the generator already has peers");
  hipError_t e = hslab_buffers(g);
  if (e != hipSuccess)
    return hip_fail(e, "ocean_peers_create: generator buffers");
  auto* p = new ocean_peers();
  p->g = g;
  p->rank = g->rank;
  p->ranks = g->ranks;
  p->slot = hslab_xbuf_bytes(g);
  p->blk = p->slot / g->ranks;
  e = hipMalloc(&p->data, 2 * p->slot);
  // the flag words in uncached memory: polled by one wave, written by the peers over xGMI
  if (e == hipSuccess)
  {
    if (hipExtMallocWithFlags((void**)&p->flags, kFlagWords * sizeof(uint32_t), hipDeviceMallocUncached) == hipSuccess)
      p->flags_uncached = true;
    else
    {
      (void)hipGetLastError();
      e = hipMalloc(&p->flags, kFlagWords * sizeof(uint32_t));
    }
  }
  if (e == hipSuccess)
    e = hipMalloc(&p->table, 3 * kMaxRanks * sizeof(uint64_t));
  if (e == hipSuccess)
    e = hipMemset(p->flags, 0, kFlagWords * sizeof(uint32_t));
  for (int k = 0; k < 2 && e == hipSuccess; k++)
  {
    e = hipEventCreateWithFlags(&p->s1_done[k], hipEventDisableTiming);
    if (e == hipSuccess)
      e = hipEventCreateWithFlags(&p->put_done[k], hipEventDisableTiming);
  }
  if (e == hipSuccess)
    e = hipEventCreateWithFlags(&p->rows_done, hipEventDisableTiming);
  if (e == hipSuccess)
    e = hipEventCreateWithFlags(&p->gen_ready, hipEventDisableTiming);
  if (e == hipSuccess)
    e = hipDeviceSynchronize();
  int rc = e == hipSuccess ? peers_deadline(p) : OCEAN_OK;
  if (rc == OCEAN_OK && e == hipSuccess)
    rc = peers_streams(p);
  if (e != hipSuccess || rc != OCEAN_OK)
  {
    const int code = e == hipErrorOutOfMemory ? OCEAN_ERR_OOM : OCEAN_ERR_HIP;
    p->g = nullptr;
    ocean_peers_destroy(p);
    return rc != OCEAN_OK ? rc : fail(code, std::string("ocean_peers_create: ") + hipGetErrorString(e));
  }
  p->peer_data[p->rank] = p->data;
  p->peer_flags[p->rank] = p->flags;
  g->peers = p;
  *out = p;
  return OCEAN_OK;
}

int ocean_peers_destroy(ocean_peers* p)
{
  if (!p)
    return OCEAN_OK;
  peers_release(p);
  if (p->g)
    p->g->peers = nullptr;
  for (hipStream_t st : {p->own_s1, p->own_put, p->own_rows})
    if (st)
      (void)hipStreamDestroy(st);
  for (int k = 0; k < 2; k++)
    for (hipEvent_t ev : {p->s1_done[k], p->put_done[k]})
      if (ev)
        (void)hipEventDestroy(ev);
  for (hipEvent_t ev : {p->rows_done, p->gen_ready})
    if (ev)
      (void)hipEventDestroy(ev);
  for (void* q : {(void*)p->data, (void*)p->flags, (void*)p->table, (void*)p->parts2})
    if (q)
      (void)hipFree(q);
  delete p;
  return OCEAN_OK;
}

int ocean_peers_handle(const ocean_peers* p, unsigned char handle[OCEAN_PEER_HANDLE_BYTES])
{
  if (!p || !handle)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_handle: null argument");
  PeerHandle h{};
  h.magic = kPeerMagic;
  h.rank = p->rank;
  h.ranks = p->ranks;
  h.flags_uncached = p->flags_uncached ? 1 : 0;
  h.slot_bytes = p->slot;
  HIP_TRY(hipIpcGetMemHandle(&h.data, p->data), "ocean_peers_handle: hipIpcGetMemHandle (slots)");
  HIP_TRY(hipIpcGetMemHandle(&h.flags, p->flags), "ocean_peers_handle: hipIpcGetMemHandle (flags)");
  std::memset(handle, 0, OCEAN_PEER_HANDLE_BYTES);
  std::memcpy(handle, &h, sizeof(h));
  return OCEAN_OK;
}

int ocean_peers_connect(ocean_peers* p, const unsigned char* handles)
{
  if (!p || !handles || !p->g)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_connect: null argument or detached peers");
  if (p->connected)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_connect: already connected");
  for (int q = 0; q < p->ranks; q++)
  {
    PeerHandle h;
    std::memcpy(&h, handles + (size_t)q * OCEAN_PEER_HANDLE_BYTES, sizeof(h));
    if (h.magic != kPeerMagic || h.rank != q || h.ranks != p->ranks || h.slot_bytes != p->slot)
      return fail(OCEAN_ERR_INVALID, "ocean_peers_connect: handle " + std::to_string(q) + " is not rank " +
                                         std::to_string(q) + " of " + std::to_string(p->ranks) +
                                         " with this grid's slot size");
    if (q == p->rank)
      continue;
    void* d = nullptr;
    void* fl = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&d, h.data, hipIpcMemLazyEnablePeerAccess);
    if (e == hipSuccess)
    {
      p->peer_data[q] = static_cast<unsigned char*>(d);
      p->mapped[q] = true;
      e = hipIpcOpenMemHandle(&fl, h.flags, hipIpcMemLazyEnablePeerAccess);
    }
    if (e == hipSuccess)
    {
      p->peer_flags[q] = static_cast<uint32_t*>(fl);
      p->mapped[kMaxRanks + q] = true;
    }
    if (e != hipSuccess)
    {
      peers_release(p);
      return hip_fail(e, ("ocean_peers_connect: hipIpcOpenMemHandle of rank " + std::to_string(q)).c_str());
    }
  }
  return peers_table(p);
}

int ocean_peers_connect_local(ocean_peers* const* all, int ranks)
{
  if (!all || ranks < 1 || ranks > kMaxRanks)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_connect_local: null array or ranks outside [1, 16]");
  for (int q = 0; q < ranks; q++)
    if (!all[q] || !all[q]->g || all[q]->rank != q || all[q]->ranks != ranks || all[q]->slot != all[0]->slot ||
        all[q]->connected)
      return fail(OCEAN_ERR_INVALID, "ocean_peers_connect_local: entry " + std::to_string(q) +
                                         " is not an unconnected rank " + std::to_string(q) + " of " +
                                         std::to_string(ranks) + " of one grid");
  for (int r = 0; r < ranks; r++)
  {
    for (int q = 0; q < ranks; q++)
    {
      all[r]->peer_data[q] = all[q]->data;
      all[r]->peer_flags[q] = all[q]->flags;
    }
    const int rc = peers_table(all[r]);
    if (rc != OCEAN_OK)
      return rc;
  }
  return OCEAN_OK;
}

int ocean_peers_set_timeout(ocean_peers* p, int ms)
{
  if (!p || ms < 1)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_set_timeout: null peers or ms < 1");
  p->timeout_ms = ms;
  return peers_deadline(p);
}

int ocean_peers_set_put_cus(ocean_peers* p, int cus)
{
  if (!p || !p->g || cus < 0 || cus > p->g->fft->device_cus)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_set_put_cus: null peers or CUs outside [0, device CUs]");
  p->put_cus = cus;
  return OCEAN_OK;
}

int ocean_peers_set_streams(ocean_peers* p, void* column_stream, void* put_stream, void* row_stream)
{
  if (!p || !p->g)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_set_streams: null or detached peers");
  if (p->rows < p->frames)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_set_streams: a pipelined frame is in flight (flush first)");
  for (hipStream_t st : {p->s1_stream, p->put_stream, p->row_stream})
    HIP_TRY(hipStreamSynchronize(st), "ocean_peers_set_streams");
  p->s1_stream = column_stream ? (hipStream_t)column_stream : p->own_s1;
  p->put_stream = put_stream ? (hipStream_t)put_stream : p->own_put;
  p->row_stream = row_stream ? (hipStream_t)row_stream : p->own_rows;
  p->put_done_valid[0] = p->put_done_valid[1] = false;  // the old streams are drained
  return OCEAN_OK;
}

int ocean_peers_set_row_cus(ocean_peers* p, int cus)
{
  if (!p || !p->g || cus < 0)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_set_row_cus: null peers or negative CUs");
  p->caller_row_cus = cus;
  return OCEAN_OK;
}

int ocean_peers_set_put_cu_mask(ocean_peers* p, int cus_per_xcd)
{
  if (!p || !p->g || cus_per_xcd < 0 || cus_per_xcd >= p->g->fft->device_cus / 8)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_set_put_cu_mask: null peers or CUs per XCD outside [0, CUs / 8)");
  if (p->rows < p->frames)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_set_put_cu_mask: a pipelined frame is in flight (flush first)");
  const bool own = p->s1_stream == p->own_s1 && p->put_stream == p->own_put && p->row_stream == p->own_rows;
  if (!own)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_set_put_cu_mask: the caller's streams are in use (ocean_peers_set_streams)");
  p->put_cus_per_xcd = cus_per_xcd;
  return peers_streams(p);
}

int ocean_generator_slab_put_columns(ocean_generator* g, ocean_peers* p, float timestep, int update_spectrum)
{
  int rc = check_peers(g, p, "ocean_generator_slab_put_columns");
  if (rc == OCEAN_OK && g->pending_slot >= 0)
    rc = ocean_generator_slab_flush(g);  // an RCCL pipelined frame in flight lands first
  return rc != OCEAN_OK ? rc : put_columns(g, p, timestep, update_spectrum, false);
}

int ocean_generator_slab_put_rows(ocean_generator* g, ocean_peers* p)
{
  const int rc = check_peers(g, p, "ocean_generator_slab_put_rows");
  return rc != OCEAN_OK ? rc : put_rows(g, p);
}

int ocean_generator_slab_frame_put(ocean_generator* g, ocean_peers* p, float timestep, int update_spectrum)
{
  int rc = check_peers(g, p, "ocean_generator_slab_frame_put");
  if (rc == OCEAN_OK && g->pending_slot >= 0)
    rc = ocean_generator_slab_flush(g);
  while (rc == OCEAN_OK && p->rows < p->frames)  // a pipelined frame in flight lands first
    rc = put_rows(g, p);
  if (rc == OCEAN_OK)
    rc = put_columns(g, p, timestep, update_spectrum, false);
  return rc != OCEAN_OK ? rc : put_rows(g, p);
}

int ocean_generator_slab_frame_put_pipelined(ocean_generator* g, ocean_peers* p, float timestep, int update_spectrum)
{
  int rc = check_peers(g, p, "ocean_generator_slab_frame_put_pipelined");
  if (rc == OCEAN_OK && g->pending_slot >= 0)
    rc = ocean_generator_slab_flush(g);
  if (rc == OCEAN_OK)
    rc = put_columns(g, p, timestep, update_spectrum, true);
  while (rc == OCEAN_OK && p->rows < p->frames - 1)  // frame f - 1's row pass beside frame f's columns
    rc = put_rows(g, p, true);
  return rc;
}

int ocean_peers_flush(ocean_peers* p)
{
  if (!p || !p->g)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_flush: null or detached peers");
  int rc = OCEAN_OK;
  while (rc == OCEAN_OK && p->rows < p->frames)
    rc = put_rows(p->g, p, true);
  return rc;
}

int ocean_peers_synchronize(ocean_peers* p)
{
  if (!p)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_synchronize: null peers");
  HIP_TRY(hipStreamSynchronize(p->s1_stream), "ocean_peers_synchronize: column stream");
  HIP_TRY(hipStreamSynchronize(p->put_stream), "ocean_peers_synchronize: put stream");
  HIP_TRY(hipStreamSynchronize(p->row_stream), "ocean_peers_synchronize: row stream");
  if (p->g)
    HIP_TRY(hipStreamSynchronize(p->g->fft->stream), "ocean_peers_synchronize: generator stream");
  uint32_t err = 0;
  HIP_TRY(hipMemcpy(&err, p->flags + kErrWord, sizeof(err), hipMemcpyDeviceToHost), "ocean_peers_synchronize: status");
  if (err != 0)
  {
    // The word is sticky on the device (every later wait returns at once). Now that the streams are
    // drained it is cleared, and the peers refuse further frames (check_peers): after a timeout the
    // ranks' ready / freed counts no longer agree, so the only way on is a new peers object.
    p->failed = true;
    HIP_TRY(hipMemset(p->flags + kErrWord, 0, sizeof(uint32_t)), "ocean_peers_synchronize: clear status");
    HIP_TRY(hipDeviceSynchronize(), "ocean_peers_synchronize: clear status");
    return fail(OCEAN_ERR_TIMEOUT, std::string("one-sided exchange: a wait for the peers' ") +
                                       (err - 1 == kReadyWord ? "blocks (ready)" : "slot release (freed)") +
                                       " timed out after " + std::to_string(p->timeout_ms) +
                                       " ms; the frames since then are invalid, and this peers object refuses new "
                                       "frames");
  }
  return p->failed ? fail(OCEAN_ERR_TIMEOUT, "one-sided exchange: an earlier wait timed out; recreate the peers")
                   : OCEAN_OK;
}

int ocean_peers_debug_slot(const ocean_peers* p, int slot, void** ptr, size_t* bytes)
{
  if (!p || !ptr || !bytes || slot < 0 || slot > 1)
    return fail(OCEAN_ERR_INVALID, "ocean_peers_debug_slot: null argument or slot outside {0, 1}");
  *ptr = p->data + (size_t)slot * p->slot;
  *bytes = p->slot;
  return OCEAN_OK;
}

int ocean_slab_layout(size_t texture_size, int rank, int ranks, int half, int64_t out[6])
{
  int logn = 0;
  while (logn < 15 && ((size_t)1 << logn) < texture_size)
    logn++;
  if (!out || ((size_t)1 << logn) != texture_size || logn < 4 || logn > 14 || ranks < 1 || ranks > 16 ||
      (ranks & (ranks - 1)) != 0 || rank < 0 || rank >= ranks)
    return fail(OCEAN_ERR_INVALID, "ocean_slab_layout: N a power of two in [16, 16384], ranks a power of two <= 16");
  if (half && !half_slab_supported(logn))
    return fail(OCEAN_ERR_INVALID, "ocean_slab_layout: the half-spectrum path needs N >= 1024");
  if (half == 2 && !gen4_supported(logn))
    return fail(OCEAN_ERR_INVALID, "ocean_slab_layout: the four-step path needs N = 8192 or 16384");
  const int n = 1 << logn, w = n / ranks;
  if (half == 2)
  {
    const Gen4Geom q = gen4_geom(logn, 1, rank, ranks, ranks == 1);
    const int64_t v[6] = {q.u0, q.cols, q.nyq, q.w, (int64_t)q.blk_bytes, (int64_t)q.blk_bytes * ranks};
    std::memcpy(out, v, sizeof(v));
  }
  else if (half)
  {
    const HalfSlab h = half_slab_geom(logn, rank, ranks);
    const int64_t blk = (int64_t)half_slab_block_bytes(logn, 1, h);
    const int64_t v[6] = {h.strip0, h.nstrips, h.S, h.w, blk, blk * ranks};
    std::memcpy(out, v, sizeof(v));
  }
  else
  {
    const int64_t blk = (int64_t)2 * w * w * sizeof(float4);
    const int64_t v[6] = {(int64_t)rank * w, w, 0, w, blk, blk * ranks};
    std::memcpy(out, v, sizeof(v));
  }
  return OCEAN_OK;
}

int ocean_generator_slab_info(const ocean_generator* g, int* rank, int* ranks, int* row0, int* rows)
{
  if (!g)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_slab_info: null generator");
  if (rank)
    *rank = g->rank;
  if (ranks)
    *ranks = g->ranks;
  if (row0)
    *row0 = g->rank * g->geom.w;
  if (rows)
    *rows = g->geom.w;
  return OCEAN_OK;
}

float* ocean_generator_height_map(ocean_generator* g, int c)
{
  if (!g || c < 0 || c >= g->cascades)
    return nullptr;
  return reinterpret_cast<float*>(g->maps + (size_t)g->fft->n * g->geom.w * (2 * c));
}

float* ocean_generator_displacement_map(ocean_generator* g, int c)
{
  if (!g || c < 0 || c >= g->cascades)
    return nullptr;
  return reinterpret_cast<float*>(g->maps + (size_t)g->fft->n * g->geom.w * (2 * c + 1));
}

float* ocean_generator_jacobian_map(ocean_generator* g, int c)
{
  if (!g || c < 0 || c >= g->cascades)
    return nullptr;
  return g->jac + (size_t)g->fft->n * g->geom.w * c;
}

static int surface_params(ocean_generator* const* gens, const int* cascades, int count, SurfaceParams& p,
                          ocean_fft*& fft, const char* who)
{
  if (!gens || !cascades || count < 1 || count > kMaxSurfaceCascades)
    return fail(OCEAN_ERR_INVALID, std::string(who) + ": need 1..16 (generator, cascade) pairs");
  p = SurfaceParams{};
  p.count = count;
  fft = nullptr;
  for (int i = 0; i < count; i++)
  {
    ocean_generator* g = gens[i];
    if (!g || cascades[i] < 0 || cascades[i] >= g->cascades)
      return fail(OCEAN_ERR_INVALID, std::string(who) + ": null generator or cascade out of range");
    if (g->ranks != 1)
      return fail(OCEAN_ERR_INVALID, std::string(who) + ": slab generators hold row slabs, not whole maps");
    if (!fft)
      fft = g->fft;
    else if (g->fft->n != fft->n)
      return fail(OCEAN_ERR_INVALID, std::string(who) + ": all cascades must share one map size");
    const int c = cascades[i];
    p.c[i].height = reinterpret_cast<const float4*>(ocean_generator_height_map(g, c));
    p.c[i].disp = reinterpret_cast<const float4*>(ocean_generator_displacement_map(g, c));
    p.c[i].jac = ocean_generator_jacobian_map(g, c);
    p.c[i].plane = g->settings[c].planeSize;
    p.c[i].scale = g->settings[c].displacement;
  }
  p.n = fft->n;
  p.atlas = nullptr;
  return OCEAN_OK;
}

// The surface atlas of a request (surface_use_atlas), owned by the plan whose stream runs the request:
// requests on one plan are stream-ordered, so one buffer serves them all.
static int surface_atlas(ocean_fft* fft, SurfaceParams& p, int64_t points, const char* who)
{
  if (!surface_use_atlas(p, points))
    return OCEAN_OK;
  const size_t texels = surface_atlas_texels(p);
  if (fft->surf_atlas_texels < texels)
  {
    if (fft->surf_atlas)
    {
      HIP_TRY(hipStreamSynchronize(fft->stream), who);  // an earlier request may still read the old one
      HIP_TRY(hipFree(fft->surf_atlas), who);
      fft->surf_atlas = nullptr;
      fft->surf_atlas_texels = 0;
    }
    HIP_TRY(hipMalloc(&fft->surf_atlas, texels * sizeof(float4)), who);
    fft->surf_atlas_texels = texels;
  }
  p.atlas = fft->surf_atlas;
  return OCEAN_OK;
}

int ocean_surface_sample(ocean_generator* const* gens, const int* cascades, int count, const float* xz,
                         int64_t points, float* out)
{
  SurfaceParams p;
  ocean_fft* fft;
  int rc = surface_params(gens, cascades, count, p, fft, "ocean_surface_sample");
  if (rc != OCEAN_OK)
    return rc;
  if (points < 0 || (points > 0 && (!xz || !out)))
    return fail(OCEAN_ERR_INVALID, "ocean_surface_sample: null positions/output or negative count");
  rc = surface_atlas(fft, p, points, "ocean_surface_sample");
  if (rc != OCEAN_OK)
    return rc;
  HIP_TRY(launch_surface(p, SurfacePlane{}, reinterpret_cast<const float2*>(xz), points, reinterpret_cast<float4*>(out),
                         fft->stream, fft->cus),
          "ocean_surface_sample");
  return OCEAN_OK;
}

int ocean_surface_sample_plane(ocean_generator* const* gens, const int* cascades, int count, const float camera[5],
                               int res, float* out)
{
  SurfaceParams p;
  ocean_fft* fft;
  int rc = surface_params(gens, cascades, count, p, fft, "ocean_surface_sample_plane");
  if (rc != OCEAN_OK)
    return rc;
  if (!camera || !out || res < 1 || res > 46340)
    return fail(OCEAN_ERR_INVALID, "ocean_surface_sample_plane: null camera/output or resolution outside 1..46340");
  if (camera[3] == 0.0f && camera[4] == 0.0f)
    return fail(OCEAN_ERR_INVALID, "ocean_surface_sample_plane: camera forward has no horizontal component");
  const SurfacePlane plane{res, camera[0], camera[1], camera[2], camera[3], camera[4]};
  const int64_t pts = (int64_t)(res + 1) * (res + 1);
  rc = surface_atlas(fft, p, pts, "ocean_surface_sample_plane");
  if (rc != OCEAN_OK)
    return rc;
  HIP_TRY(launch_surface(p, plane, nullptr, pts, reinterpret_cast<float4*>(out), fft->stream, fft->cus),
          "ocean_surface_sample_plane");
  return OCEAN_OK;
}

float* ocean_generator_initial_spectrum(ocean_generator* g, int c)
{
  if (!g || c < 0 || c >= g->cascades)
    return nullptr;
  if (materialise_h0(g) != OCEAN_OK)  // after fused re-seed frames
    return nullptr;
  // the caller may write h0 through this pointer: the next requested re-seed must regenerate it, as
  // the reference does on every request (src/Generator.cpp:55-59), so the h0 memo forgets its inputs
  g->seeded.clear();
  g->h0_dirty = true;  // frame overlap: the next column pass waits for the caller's stream (its h0 writes)
  return reinterpret_cast<float*>(g->h0 + h0_texels(g) * c);
}

int ocean_generator_spectrum_block(const ocean_generator* g)
{
  return g ? (g->h0_block > 0 ? g->h0_block : h0_block(g)) : 0;  // the layout h0 holds now
}

int ocean_generator_set_profiling(ocean_generator* g, int enable)
{
  if (!g)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_set_profiling: null generator");
  g->profiling = enable != 0;
  return OCEAN_OK;
}

int ocean_generator_kernel_times4(ocean_generator* g, double ms_total[4], int64_t launches[4])
{
  if (!g)
    return fail(OCEAN_ERR_INVALID, "ocean_generator_kernel_times: null generator");
  HIP_TRY(hipStreamSynchronize(g->fft->stream), "hipStreamSynchronize");
  for (auto& p : g->pending)
  {
    float ms = 0.0f;
    HIP_TRY(hipEventSynchronize(p.b), "hipEventSynchronize");  // pairs on the put stream too
    HIP_TRY(hipEventElapsedTime(&ms, p.a, p.b), "hipEventElapsedTime");
    g->ms[p.kind] += ms;
    g->launches[p.kind] += 1;
    g->pool.push_back(p.a);
    g->pool.push_back(p.b);
  }
  g->pending.clear();
  for (int k = 0; k < 4; k++)
  {
    if (ms_total)
      ms_total[k] = g->ms[k];
    if (launches)
      launches[k] = g->launches[k];
    g->ms[k] = 0;
    g->launches[k] = 0;
  }
  return OCEAN_OK;
}

int ocean_generator_kernel_times(ocean_generator* g, double ms_total[3], int64_t launches[3])
{
  double m[4];
  int64_t l[4];
  const int rc = ocean_generator_kernel_times4(g, m, l);
  for (int k = 0; rc == OCEAN_OK && k < 3; k++)
  {
    if (ms_total)
      ms_total[k] = m[k];
    if (launches)
      launches[k] = l[k];
  }
  return rc;
}

int ocean_debug_copy(void* dst, const void* src, size_t bytes, int workgroups, void* hip_stream)
{
  if ((bytes > 0 && (!dst || !src)) || bytes % 16 != 0 || workgroups < 1 || workgroups > 65536 ||
      (reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) % 16 != 0)
    return fail(OCEAN_ERR_INVALID, "ocean_debug_copy: null or unaligned pointer, bytes not a multiple of 16, or "
                                   "workgroups outside [1, 65536]");
  if (bytes == 0)
    return OCEAN_OK;
  HIP_TRY(launch_debug_copy(dst, src, bytes, workgroups, (hipStream_t)hip_stream), "debug copy");
  return OCEAN_OK;
}

int ocean_debug_hash(const uint32_t* xy, int count, uint32_t* raw, float* uv, void* hip_stream)
{
  if (!xy || !raw || !uv || count < 0)
    return fail(OCEAN_ERR_INVALID, "ocean_debug_hash: null argument");
  if (count == 0)
    return OCEAN_OK;
  HIP_TRY(launch_hash(xy, count, raw, reinterpret_cast<float2*>(uv), (hipStream_t)hip_stream), "hash");
  return OCEAN_OK;
}

}  // extern "C"
