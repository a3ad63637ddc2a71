/*
 * ocean_oracle.c — CPU restatement of the reference ocean hot path (TEST INFRASTRUCTURE ONLY).
 *
 * Not shipped, not measured as the product: tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg are the only users. Parity is UNPINNED by reference outputs (the reference has
 * no tests/fixtures and its GLSL path cannot run here) — see ocean_oracle.h and DESIGN.md.
 *
 * Semantics follow the GLSL exactly in float32: every literal is a float literal, every operation
 * is evaluated left to right as written, no FMA contraction (built with -ffp-contract=off), and the
 * transcendentals are the C library's float functions. GLSL's pow/exp/tanh on the author's GPU are
 * lower precision than libm; that difference is what the parity tolerances absorb.
 */
#include "ocean_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* resources/spectrum.compute:4 and resources/fft.compute:14 — both round to the same float. */
#define PI_SPECTRUM 3.14159265358f
#define PI_FFT 3.141592653589793238f

/* resources/spectrum.compute:34-35 */
static const float SIGMA_SURFACE = 0.072f;
static const float RHO_WATER = 1000.0f;

static int g_threads = 1;

void oracle_set_threads(int threads)
{
  g_threads = threads < 1 ? 1 : threads;
}

int oracle_get_threads(void)
{
#ifdef _OPENMP
  return g_threads;
#else
  return 1;
#endif
}

/* src/Generator.h:14-29 */
void oracle_default_settings(oracle_settings* s)
{
  memset(s, 0, sizeof(*s));
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

/* resources/spectrum.compute:38-44 */
static float dispersion(const oracle_settings* s, float k)
{
  float kh = k * s->h;
  float tanhKH = kh >= 2.0f * PI_SPECTRUM ? 1.0f : tanhf(kh);
  float omegaSquared = (s->g * k + SIGMA_SURFACE / RHO_WATER * k * k * k) * tanhKH;
  return sqrtf(omegaSquared);
}

/* resources/spectrum.compute:50-57 */
static float dispersion_derivative(const oracle_settings* s, float k)
{
  float phi = dispersion(s, k);
  float sech = 1.0f / coshf(s->h * k);
  float numerator = s->h * (SIGMA_SURFACE / RHO_WATER * k * k * k + s->g * k) * sech * sech + phi * phi;
  return numerator / (2.0f * phi);
}

/* GLSL smoothstep(edge0, edge1, x) */
static float smoothstep_f(float e0, float e1, float x)
{
  float t = (x - e0) / (e1 - e0);
  t = t < 0.0f ? 0.0f : (t > 1.0f ? 1.0f : t);
  return t * t * (3.0f - 2.0f * t);
}

/* resources/spectrum.compute:60-78 */
static float jonswap(const oracle_settings* s, float k, float omega, float omega_p)
{
  (void)k;
  float alpha = 0.076f * powf(s->U_10 * s->U_10 / (s->F * s->g), 0.22f);
  float gamma = 3.3f;
  float sigma = omega > omega_p ? 0.09f : 0.07f;

  float omegaDiff = fabsf(omega - omega_p);
  float omegaRatio = omega_p / omega;
  float r = expf(-omegaDiff * omegaDiff / (2.0f * sigma * sigma * omega_p * omega_p));
  float S = alpha * s->g * s->g / powf(omega, 5.0f) * expf(-1.25f * powf(omegaRatio, 4.0f)) *
            powf(gamma, r);

  float w_h = fminf(omega * sqrtf(s->h / s->g), 2.0f);
  float kit = smoothstep_f(0.0f, 2.2f, w_h);
  return S * kit;
}

/* resources/spectrum.compute:81-88 */
static float lh_normalization(float s)
{
  float a = sqrtf(s);
  return (s < 0.4f) ? (0.5f / PI_SPECTRUM) + s * (0.220636f + s * (-0.109f + s * 0.090f))
                    : (1.0f / sqrtf(PI_SPECTRUM)) * (a * 0.5f + (1.0f / a) * 0.0625f);
}

/* resources/spectrum.compute:91-94 */
static float lh_function(float s, float theta)
{
  return lh_normalization(s) * powf(fabsf(cosf(theta * 0.5f)), 2.0f * s);
}

/* resources/spectrum.compute:97-106 */
static float hasselmann(const oracle_settings* st, float w, float w_p, float wind_speed, float theta)
{
  float p = w / w_p;
  float s = (w <= w_p) ? 6.97f * powf(fabsf(p), 4.06f)
                       : 9.77f * powf(fabsf(p), -2.33f - 1.45f * (wind_speed * w_p / st->g - 1.17f));
  float s_xi = 16.0f * tanhf(w_p / w) * st->swell * st->swell;
  return lh_function(s + s_xi, theta);
}

/* resources/spectrum.compute:109-117 */
void oracle_hash(uint32_t x, uint32_t y, float out[2], uint32_t* raw)
{
  uint32_t h32 = y + 374761393u + x * 3266489917u;
  h32 = 2246822519u * (h32 ^ (h32 >> 15));
  h32 = 3266489917u * (h32 ^ (h32 >> 13));
  uint32_t n = h32 ^ (h32 >> 16);
  uint32_t rz0 = n, rz1 = n * 48271u;
  out[0] = (float)((rz0 >> 1) & 0x7FFFFFFFu) / (float)0x7FFFFFFF;
  out[1] = (float)((rz1 >> 1) & 0x7FFFFFFFu) / (float)0x7FFFFFFF;
  if (raw)
    *raw = n;
}

/* resources/spectrum.compute:121-127 */
static void gaussian(const float u[2], float out[2])
{
  float r = sqrtf(-2.0f * logf(u[0]));
  float theta = 2.0f * PI_SPECTRUM * u[1];
  out[0] = r * cosf(theta);
  out[1] = r * sinf(theta);
}

/* GLSL uint(float) for the non-negative values the seeds produce (spectrum.compute:153). */
static uint32_t to_uint(float v)
{
  return (uint32_t)(int64_t)v;
}

/* resources/spectrum.compute:129-155 */
void oracle_spectrum_amplitude(const oracle_settings* s, float tx, float ty, float dimx, float dimy,
                               float out[2])
{
  float dk = 2.0f * PI_SPECTRUM / s->planeSize;
  float kx = (tx - dimx / 2.0f) * dk;
  float ky = (ty - dimy / 2.0f) * dk;
  float k = sqrtf(kx * kx + ky * ky);
  float theta = atan2f(ky, kx) - s->theta_0;

  if (k == 0.0f)
  {
    out[0] = 0.0f;
    out[1] = 0.0f;
    return;
  }

  float omega = dispersion(s, k);
  float omega_p = 22.0f * powf(s->g * s->g / (s->U_10 * s->F), 0.333f);

  float Sj = jonswap(s, k, omega, omega_p);
  float d = ((1.0f - s->spread) * hasselmann(s, omega, omega_p, s->U_10, theta) +
             (s->spread) / (2.0f * PI_SPECTRUM));

  float chain = dispersion_derivative(s, k) / k * dk * dk;

  float u[2], gs[2];
  oracle_hash(to_uint(tx + (float)s->seed[0]), to_uint(ty + (float)s->seed[1]), u, NULL);
  gaussian(u, gs);
  float amp = sqrtf(2.0f * Sj * d * chain);
  float c = 0.1f * s->scale;
  out[0] = c * gs[0] * amp;
  out[1] = c * gs[1] * amp;
}

/* resources/spectrum.compute:157-172 */
void oracle_generate_spectrum(const oracle_settings* s, int n, float* h0)
{
  const float dim = (float)n;
#pragma omp parallel for num_threads(g_threads) schedule(static)
  for (int y = 0; y < n; y++)
  {
    for (int x = 0; x < n; x++)
    {
      float a[2], b[2];
      oracle_spectrum_amplitude(s, (float)x, (float)y, dim, dim, a);
      oracle_spectrum_amplitude(s, dim - (float)x, dim - (float)y, dim, dim, b);
      float* o = h0 + 4 * ((size_t)y * n + x);
      o[0] = a[0];
      o[1] = a[1];
      o[2] = b[0];
      o[3] = -b[1];
    }
  }
}

/* resources/spectrum.compute:157-172 at `count` texels (x, y) of an N x N image (the same
   per-texel body as oracle_generate_spectrum): sampled checks at sizes where the whole image
   would take the oracle minutes (N = 16384). xy: count int32 pairs; h0: count float4. */
void oracle_spectrum_texels(const oracle_settings* s, int n, int64_t count, const int32_t* xy, float* h0)
{
  const float dim = (float)n;
#pragma omp parallel for num_threads(g_threads) schedule(static)
  for (int64_t i = 0; i < count; i++)
  {
    float a[2], b[2];
    float x = (float)xy[2 * i], y = (float)xy[2 * i + 1];
    oracle_spectrum_amplitude(s, x, y, dim, dim, a);
    oracle_spectrum_amplitude(s, dim - x, dim - y, dim, dim, b);
    float* o = h0 + 4 * i;
    o[0] = a[0];
    o[1] = a[1];
    o[2] = b[0];
    o[3] = -b[1];
  }
}

/* resources/spectrum.compute:183-240 on the spectrum rows [y0, y0 + rows); h0, height, disp hold
 * those rows only (rows * N float4 each). */
void oracle_prepare_fft_rows(const oracle_settings* s, int n, int y0, int rows, const float* h0, float* height,
                             float* disp)
{
  const float dim = (float)n;
#pragma omp parallel for num_threads(g_threads) schedule(static)
  for (int r = 0; r < rows; r++)
  {
    const int y = y0 + r;
    for (int x = 0; x < n; x++)
    {
      float dk = 2.0f * PI_SPECTRUM / s->planeSize;
      float kx = ((float)x - dim / 2.0f) * dk;
      float kz = ((float)y - dim / 2.0f) * dk;
      float len = sqrtf(kx * kx + kz * kz);
      float dirx = 0.0f, dirz = 0.0f;
      if (!(kx == 0.0f && kz == 0.0f))
      {
        dirx = kx / len;
        dirz = kz / len;
      }
      float k = len + 1e-6f;

      const float* a = h0 + 4 * ((size_t)r * n + x);
      float phase = dispersion(s, k) * s->time;
      float wc = cosf(phase), ws = sinf(phase);

      /* ComplexMultiply(amplitude, wave), spectrum.compute:29-32 */
      float ampx = a[0] * wc - a[1] * ws;
      float ampy = a[0] * ws + a[1] * wc;
      /* wave.y *= -1 */
      float ws2 = -ws;
      float oppx = a[2] * wc - a[3] * ws2;
      float oppy = a[2] * ws2 + a[3] * wc;

      float hx = ampx + oppx, hy = ampy + oppy;
      float ihx = -hy, ihy = hx; /* heightAmpTimesi */

      float dhdx_x = kx * (-hy), dhdx_y = kx * hx;
      float dhdz_x = kz * (-hy), dhdz_y = kz * hx;
      float disX_x = dirx * ihx, disX_y = dirx * ihy;
      float disZ_x = dirz * ihx, disZ_y = dirz * ihy;
      float dDXdx_x = -kx * dirx * hx, dDXdx_y = -kx * dirx * hy;
      float dDZdz_x = -kz * dirz * hx, dDZdz_y = -kz * dirz * hy;
      float dDXdz_x = -kz * dirx * hx, dDXdz_y = -kz * dirx * hy;

      float* o0 = height + 4 * ((size_t)r * n + x);
      float* o1 = disp + 4 * ((size_t)r * n + x);
      o0[0] = hx - dhdx_y;
      o0[1] = hy + dhdx_x;
      o0[2] = dhdz_x - disX_y;
      o0[3] = dhdz_y + disX_x;
      o1[0] = disZ_x - dDXdx_y;
      o1[1] = disZ_y + dDXdx_x;
      o1[2] = dDZdz_x - dDXdz_y;
      o1[3] = dDZdz_y + dDXdz_x;
    }
  }
}

/* resources/spectrum.compute:183-240 */
void oracle_prepare_fft(const oracle_settings* s, int n, const float* h0, float* height, float* disp)
{
  oracle_prepare_fft_rows(s, n, 0, n, h0, height, disp);
}

/* resources/fft.compute:21-28 — out[(p + SIZE/2) % SIZE] = in[p] on both axes. */
static void fft_shift(int n, const float* in, float* out)
{
#pragma omp parallel for num_threads(g_threads) schedule(static)
  for (int y = 0; y < n; y++)
    for (int x = 0; x < n; x++)
    {
      int ex = (x + n / 2) % n, ey = (y + n / 2) % n;
      memcpy(out + 4 * ((size_t)ey * n + ex), in + 4 * ((size_t)y * n + x), 16);
    }
}

/* resources/fft.compute:32-35 */
static uint32_t reverse_bits(uint32_t num, uint32_t bits)
{
  uint32_t r = 0;
  for (uint32_t i = 0; i < 32; i++)
    if (num & (1u << i))
      r |= 1u << (31 - i);
  return bits == 0 ? 0 : r >> (32 - bits);
}

/* resources/fft.compute:38-48 */
static void image_reversal(int n, const float* in, float* out)
{
  uint32_t logn = 0;
  while ((1 << logn) < n)
    logn++;
#pragma omp parallel for num_threads(g_threads) schedule(static)
  for (int y = 0; y < n; y++)
    for (int x = 0; x < n; x++)
    {
      uint32_t rx = reverse_bits((uint32_t)x, logn), ry = reverse_bits((uint32_t)y, logn);
      memcpy(out + 4 * ((size_t)y * n + x), in + 4 * ((size_t)ry * n + rx), 16);
    }
}

/* resources/fft.compute:54-88 — one radix-2 DIT stage; workgroup id.y = row/column, thread = j. */
static void fft_pass(int n, int passNum, int vertical, const float* in, float* out)
{
#pragma omp parallel for num_threads(g_threads) schedule(static)
  for (int line = 0; line < n; line++)
  {
    for (int thread = 0; thread < n / 2; thread++)
    {
      uint32_t halfSize = 1u << passNum;
      uint32_t fullSize = halfSize << 1;
      int dftNum = thread / (int)halfSize;
      int dftElement = thread % (int)halfSize;
      int evenIndex = dftNum * (int)fullSize + dftElement;
      int oddIndex = evenIndex + (int)halfSize;

      size_t ep = vertical ? ((size_t)evenIndex * n + line) : ((size_t)line * n + evenIndex);
      size_t op = vertical ? ((size_t)oddIndex * n + line) : ((size_t)line * n + oddIndex);

      const float* e = in + 4 * ep;
      const float* o = in + 4 * op;

      float twiddleAngle = 2.0f * PI_FFT * (float)dftElement / (float)fullSize;
      float tc = cosf(twiddleAngle), ts = sinf(twiddleAngle);

      float ox = o[0] * tc - o[1] * ts;
      float oy = o[0] * ts + o[1] * tc;
      float oz = o[2] * tc - o[3] * ts;
      float ow = o[2] * ts + o[3] * tc;

      float* oe = out + 4 * ep;
      float* oo = out + 4 * op;
      oe[0] = e[0] + ox;
      oe[1] = e[1] + oy;
      oe[2] = e[2] + oz;
      oe[3] = e[3] + ow;
      oo[0] = e[0] - ox;
      oo[1] = e[1] - oy;
      oo[2] = e[2] - oz;
      oo[3] = e[3] - ow;
    }
  }
}

/* src/FFTCalculator.cpp:73-114 (pass table :14-23): shift, bit-reverse, then log2N row passes and
 * log2N column passes, ping-ponging image <-> work so the result lands back in image. */
void oracle_encode_ifft(int n, float* image, float* work)
{
  int logn = 0;
  while ((1 << logn) < n)
    logn++;
  int numPasses = 2 * logn;

  float* src = image;
  float* dst = work;
  float* t;

  fft_shift(n, src, dst);
  t = src, src = dst, dst = t;
  image_reversal(n, src, dst);
  t = src, src = dst, dst = t;
  for (int i = 0; i < numPasses; i++)
  {
    int passNumber = i % (numPasses / 2);
    int vertical = i >= (numPasses / 2) ? 1 : 0;
    fft_pass(n, passNumber, vertical, src, dst);
    t = src, src = dst, dst = t;
  }
  /* 2 + 2*log2N swaps is even: the result is back in image (src == image). */
}

/* resources/spectrum.compute:246-259 */
void oracle_compute_foam(const oracle_settings* s, int n, const float* disp, float* jac)
{
#pragma omp parallel for num_threads(g_threads) schedule(static)
  for (int y = 0; y < n; y++)
    for (int x = 0; x < n; x++)
    {
      const float* d = disp + 4 * ((size_t)y * n + x);
      float dDxdx = d[1], dDzdz = d[2], dDxdz = d[3];
      float lam = s->displacement;
      jac[(size_t)y * n + x] =
          (1.0f + lam * dDxdx) * (1.0f + lam * dDzdz) - lam * lam * dDxdz * dDxdz;
    }
}

/* src/Generator.cpp:45-83 */
void oracle_calculate_ocean(oracle_settings* s, int n, float timestep, int update_spectrum,
                            float* h0, float* height, float* disp, float* jac, float* work)
{
  s->time += timestep;
  if (update_spectrum)
    oracle_generate_spectrum(s, n, h0);
  oracle_prepare_fft(s, n, h0, height, disp);
  oracle_encode_ifft(n, height, work);
  oracle_encode_ifft(n, disp, work);
  oracle_compute_foam(s, n, disp, jac);
}

/* ---- Surface consumer (resources/waveShader.glsl) -------------------------------------------- */

/* GL_LINEAR + GL_REPEAT on an N*N texture with `ch` channels (OpenGL 4.5 §8.14.2): texel-space
 * s = u*N - 1/2, i0 = floor(s), alpha = frac(s); weights in the specification's order. */
static void sample_bilinear(const float* tex, int n, int ch, float u, float v, float* out)
{
  float s = u * (float)n - 0.5f, t = v * (float)n - 0.5f;
  float fs = floorf(s), ft = floorf(t);
  float a = s - fs, b = t - ft;
  int i0 = (int)fs, j0 = (int)ft;
  int i0w = ((i0 % n) + n) % n, j0w = ((j0 % n) + n) % n;
  int i1w = (i0w + 1) % n, j1w = (j0w + 1) % n;
  float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
  const float* t00 = tex + ((size_t)j0w * n + i0w) * ch;
  const float* t10 = tex + ((size_t)j0w * n + i1w) * ch;
  const float* t01 = tex + ((size_t)j1w * n + i0w) * ch;
  const float* t11 = tex + ((size_t)j1w * n + i1w) * ch;
  for (int k = 0; k < ch; k++)
    out[k] = w00 * t00[k] + w10 * t10[k] + w01 * t01[k] + w11 * t11[k];
}

void oracle_surface_vertex(const oracle_cascade_maps* c, int count, float x, float z, float out[8])
{
  float px = x, py = 0.0f, pz = z;
  /* vertex stage, waveShader.glsl:101-110: each cascade samples at the position the previous
   * cascades already displaced */
  for (int i = 0; i < count; i++)
  {
    float d1[4], d2[4];
    float u = px / c[i].planeSize, v = pz / c[i].planeSize;
    sample_bilinear(c[i].height, c[i].n, 4, u, v, d1);
    sample_bilinear(c[i].disp, c[i].n, 4, u, v, d2);
    px += c[i].displacement * d1[3];
    py += d1[0];
    pz += c[i].displacement * d2[0];
  }
  /* fragment stage at the displaced position, waveShader.glsl:127-144 */
  float d[4] = {0.0f, 0.0f, 0.0f, 0.0f}, jac = 0.0f;
  for (int i = 0; i < count; i++)
  {
    float d1[4], d2[4], j;
    float u = px / c[i].planeSize, v = pz / c[i].planeSize;
    sample_bilinear(c[i].height, c[i].n, 4, u, v, d1);
    sample_bilinear(c[i].disp, c[i].n, 4, u, v, d2);
    sample_bilinear(c[i].jac, c[i].n, 1, u, v, &j);
    jac += j / (float)count; /* the reference's "/ 3.0" for its three cascades */
    float f = c[i].displacement;
    d[0] += d1[1];
    d[1] += d2[1] * f;
    d[2] += d1[2];
    d[3] += d2[2] * f;
  }
  float sx = d[0] / (1.0f + d[1]), sz = d[2] / (1.0f + d[3]);
  float nx = -sx, ny = 1.0f, nz = -sz;
  float len = sqrtf(nx * nx + ny * ny + nz * nz);
  out[0] = px;
  out[1] = py;
  out[2] = pz;
  out[3] = jac;
  out[4] = nx / len;
  out[5] = ny / len;
  out[6] = nz / len;
  out[7] = 0.0f;
}

void oracle_surface_plane(const oracle_cascade_maps* c, int count, const float cam[5], int res, float* out)
{
  /* turnDir = normalize(forward.xz), rotated by 45 degrees (waveShader.glsl:84-88) */
  float fl = sqrtf(cam[3] * cam[3] + cam[4] * cam[4]);
  float tx0 = cam[3] / fl, tz0 = cam[4] / fl;
  float tx = (tx0 - tz0) * 0.70711f, tz = (tx0 + tz0) * 0.70711f;
  float cam_y = cam[1] > 10.0f ? cam[1] : 10.0f;
  const int side = res + 1;
#pragma omp parallel for num_threads(g_threads) schedule(static)
  for (int j = 0; j < side; j++)
    for (int i = 0; i < side; i++)
    {
      /* plane vertex (src/Renderer.cpp:18), then pos + (15, 0, 15) (waveShader.glsl:77) */
      float x = -20.0f + 40.0f * (float)i / (float)res + 15.0f;
      float z = -20.0f + 40.0f * (float)j / (float)res + 15.0f;
      float rx = tx * x - tz * z, rz = x * tz + z * tx;
      float len = sqrtf(rx * rx + rz * rz);
      float k = powf(len > 1.0f ? len : 1.0f, 1.2f) * cam_y * 0.04f; /* shader's left-to-right order */
      rx = rx * k + cam[0];
      rz = rz * k + cam[2];
      oracle_surface_vertex(c, count, rx, rz, out + 8 * ((size_t)j * side + i));
    }
}

void oracle_surface_points(const oracle_cascade_maps* c, int count, const float* xz, int64_t npts, float* out)
{
#pragma omp parallel for num_threads(g_threads) schedule(static)
  for (int64_t p = 0; p < npts; p++)
    oracle_surface_vertex(c, count, xz[2 * p], xz[2 * p + 1], out + 8 * p);
}
