/*
 * ocean_oracle.h — CPU restatement of the reference ocean hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity checker and the CPU baseline for oceansimulation_amd. It is NOT part of the
 * product: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Parity status: UNPINNED by reference outputs. The reference (James51332/OceanSimulation) has no
 * tests, fixtures or golden vectors, and its path is GLSL executed through the absent Vision engine,
 * so it cannot run in this container. The restatement is cross-checked instead against an
 * independently written numpy formulation (tests/golden/make_golden.py) and analytic FFT
 * known-answer tests (tests/test_oracle.py). See DESIGN.md §Oracle.
 *
 * Every function cites the reference file:line it restates (paths relative to the reference root).
 */
#ifndef OCEAN_ORACLE_H
#define OCEAN_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same 64-byte layout as Waves::GeneratorSettings (src/Generator.h:12-30) and the std140
 * spectrumSettings UBO (resources/spectrum.compute:10-27). */
typedef struct oracle_settings
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
} oracle_settings;

/* Defaults of src/Generator.h:14-29. */
void oracle_default_settings(oracle_settings* s);

/* resources/spectrum.compute:109-117 — returns the two uniforms; raw gets the uint32 n (may be 0). */
void oracle_hash(uint32_t x, uint32_t y, float out[2], uint32_t* raw);

/* resources/spectrum.compute:129-155 for one (thread, dimensions) pair. */
void oracle_spectrum_amplitude(const oracle_settings* s, float tx, float ty, float dimx, float dimy,
                               float out[2]);

/* resources/spectrum.compute:157-172 over the whole N x N image. h0: N*N float4 (row-major, x fastest). */
void oracle_generate_spectrum(const oracle_settings* s, int n, float* h0);

/* The same texels as oracle_generate_spectrum at `count` indices (x, y) (int32 pairs); h0: count float4. */
void oracle_spectrum_texels(const oracle_settings* s, int n, int64_t count, const int32_t* xy, float* h0);

/* resources/spectrum.compute:183-240. height, disp: N*N float4 each. */
void oracle_prepare_fft(const oracle_settings* s, int n, const float* h0, float* height, float* disp);
/* The same on spectrum rows [y0, y0 + rows) only: h0, height, disp hold rows * N float4 each. */
void oracle_prepare_fft_rows(const oracle_settings* s, int n, int y0, int rows, const float* h0, float* height,
                             float* disp);

/* src/FFTCalculator.cpp:73-114 with resources/fft.compute:21-88 (SIZE generalised to n).
 * In-place on image (N*N float4); work: scratch N*N float4 (the reference's workImage). */
void oracle_encode_ifft(int n, float* image, float* work);

/* resources/spectrum.compute:246-259. jac: N*N float. */
void oracle_compute_foam(const oracle_settings* s, int n, const float* disp, float* jac);

/* src/Generator.cpp:45-83 — one CalculateOcean: time += timestep (fp32), optional spectrum
 * regeneration, evolve+pack, two EncodeIFFTs, foam. work: N*N float4 scratch. */
void oracle_calculate_ocean(oracle_settings* s, int n, float timestep, int update_spectrum,
                            float* h0, float* height, float* disp, float* jac, float* work);

/* ---- Surface consumer (resources/waveShader.glsl), SURVEY §8f rank 3 --------------------------
 * One cascade's maps as the renderer binds them (src/Renderer.cpp:62-72): heightMap and
 * displacementMap RGBA32F, jacobianMap R32F, N*N row-major, sampled GL_LINEAR + GL_REPEAT
 * (src/Generator.cpp:116-119), with the cascade's planeSize and displacement (Renderer.cpp:70-71). */
typedef struct oracle_cascade_maps
{
  const float* height;
  const float* disp;
  const float* jac;
  int n;
  float planeSize;
  float displacement;
} oracle_cascade_maps;

/* Per vertex at base position (x, 0, z): the vertex stage's displacement loop over the cascades
 * (waveShader.glsl:101-110), then at the displaced position the fragment stage's slope normal and
 * Jacobian average (waveShader.glsl:127-144). out[8] = (x, y, z, jacobian, nx, ny, nz, 0). */
void oracle_surface_vertex(const oracle_cascade_maps* c, int count, float x, float z, float out[8]);

/* oracle_surface_vertex over npts base positions xz[2*p], xz[2*p+1]; out: npts * 8 floats. */
void oracle_surface_points(const oracle_cascade_maps* c, int count, const float* xz, int64_t npts, float* out);

/* The reference's plane mesh (40 m x 40 m, res x res quads, (res+1)^2 vertices, x fastest; src/
 * Renderer.cpp:18) through the camera-relative warp of waveShader.glsl:77-98 (camera position
 * cam[0..2] = viewInverse[3].xyz, forward cam[3..4] = -viewInverse[0].xz), then
 * oracle_surface_vertex. out: (res+1)^2 * 8 floats. */
void oracle_surface_plane(const oracle_cascade_maps* c, int count, const float cam[5], int res, float* out);

/* Threads used by the OpenMP loops (1 when built without OpenMP). */
void oracle_set_threads(int threads);
int oracle_get_threads(void);

#ifdef __cplusplus
}
#endif

#endif
