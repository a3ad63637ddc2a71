/*
 * oceanfft.h — C ABI of the MI355X ocean height-field library (liboceanfft.so).
 *
 * Drop-in boundary for the hot path of James51332/OceanSimulation:
 *   Waves::FFTCalculator  (src/FFTCalculator.h:11-59, src/FFTCalculator.cpp:10-114)
 *   Waves::Generator      (src/Generator.h:33-93,     src/Generator.cpp:14-154)
 *   Waves::GeneratorSettings (src/Generator.h:12-30)
 * Every entry point below cites the reference member it replaces. The C++ classes with the
 * reference's exact signatures (include/waves/Generator.h, FFTCalculator.h) are thin wrappers over this ABI; INTEGRATION.md
 * shows the ctypes/C++ bindings.
 *
 * Conventions
 *   - Plain C types only. Device buffers are `float*` into HBM: RGBA32F images are N*N float4,
 *     row-major, x fastest (image x = column, resources/fft.compute:72-73); R32F maps are N*N float.
 *   - Every function returns an int status (OCEAN_OK == 0) unless it is a getter; on failure
 *     ocean_last_error() gives a thread-local message. (The reference has no error path at all —
 *     its calls are void and misuse such as N != SIZE silently corrupts results; here misuse fails.)
 *   - One context per HIP stream: all work of an ocean_fft and of the generators bound to it is
 *     issued on the stream given at ocean_fft_create (nullptr = the default stream). Calls only
 *     enqueue work (the reference's "encode into a command buffer"); ocean_fft_synchronize waits.
 *   - Library-owned outputs are borrowed by the caller and valid until the owner is destroyed
 *     (the reference's Vision::ID handles, src/Generator.h:48-50).
 */
#ifndef OCEANFFT_H
#define OCEANFFT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OCEAN_OK 0
#define OCEAN_ERR_INVALID 1   /* bad argument (size not a power of two in [16, 16384], null, range) */
#define OCEAN_ERR_HIP 2       /* HIP runtime error (message in ocean_last_error) */
#define OCEAN_ERR_NO_DEVICE 3 /* no GPU visible */
#define OCEAN_ERR_OOM 4       /* device allocation failed */
/* OCEAN_ERR_TIMEOUT 5: see the one-sided slab exchange below */

#define OCEAN_MAX_CASCADES 64

/* Waves::GeneratorSettings (src/Generator.h:12-30); same 64-byte layout as the std140 UBO
 * spectrumSettings (resources/spectrum.compute:10-27). */
typedef struct ocean_settings
{
  int32_t seed[2];         /* seed for the hash noise */
  float U_10;              /* wind speed */
  float theta_0;           /* wind direction (the reference subtracts it from radians as-is) */
  float F;                 /* fetch */
  float g;                 /* gravity */
  float swell;             /* swell factor */
  float h;                 /* depth */
  float displacement;      /* choppiness lambda used by the Jacobian */
  float time;              /* seconds, accumulated in fp32 by calculate() */
  float planeSize;         /* metres covered by the tile */
  float scale;             /* global amplitude scale */
  float spread;            /* directional spread blend */
  int32_t boundWavelength; /* uploaded but unused by the reference (spectrum.compute:24) */
  float wavelengthMin;     /* idem */
  float wavelengthMax;     /* idem */
} ocean_settings;

typedef struct ocean_fft ocean_fft;             /* Waves::FFTCalculator */
typedef struct ocean_generator ocean_generator; /* one or more Waves::Generator cascades */

/* ---- library ---------------------------------------------------------------------------- */
const char* ocean_last_error(void);
const char* ocean_version(void);
/* GeneratorSettings default member initialisers, src/Generator.h:14-29. */
void ocean_default_settings(ocean_settings* s);
/* Number of visible GPUs (0 when none); does not create a context. */
int ocean_device_count(void);

/* ---- FFTCalculator ------------------------------------------------------------------------ */
/* FFTCalculator::FFTCalculator(RenderDevice*, size_t textureSize) — src/FFTCalculator.cpp:10-58.
 * Builds the twiddle table on the device; texture_size must be a power of two in [16, 16384]. */
int ocean_fft_create(ocean_fft** out, size_t texture_size, void* hip_stream);
/* FFTCalculator::~FFTCalculator — src/FFTCalculator.cpp:61-71. */
int ocean_fft_destroy(ocean_fft* fft);
/* FFTCalculator::GetTextureResolution — src/FFTCalculator.h:24. */
size_t ocean_fft_texture_resolution(const ocean_fft* fft);
/* FFTCalculator::EncodeIFFT(Vision::ID image) — src/FFTCalculator.cpp:73-114. In place on a
 * device RGBA32F N*N image: out = N^2 * ifft2(ifftshift(in)) on lanes xy and zw independently
 * (no normalisation, like the reference). The caller needs no work image; the plan allocates its
 * own on first use where a faster order needs one (N = 4096: column-first through up to 8 images;
 * N = 16384: rows, then a four-step column transform through an N x 2048 slab), and falls back to
 * the in-place passes when that allocation fails. */
int ocean_fft_encode_ifft(ocean_fft* fft, float* image);
/* Batched EncodeIFFT over n_images contiguous images (image i at image + i*N*N*4 floats). */
int ocean_fft_encode_ifft_batch(ocean_fft* fft, float* images, int n_images);
/* Wait for all work enqueued on the plan's stream (the reference's SubmitCommandBuffer + fence,
 * src/Waves.cpp:106). */
int ocean_fft_synchronize(ocean_fft* fft);
/* Multiprocessor (CU) count of the plan's device. */
int ocean_fft_device_cus(const ocean_fft* fft);
/* Size the plan's persistent grids (every kernel of this plan and its generators) for `cus` CUs
 * instead of all of them (0 restores all). The frame kernels take a whole CU per workgroup, so a
 * budget below the device count leaves CUs free for work on other streams, e.g. the copy kernels
 * of an RCCL all-to-all overlapped with the slab passes. No reference counterpart. */
int ocean_fft_set_cu_budget(ocean_fft* fft, int cus);

/* ---- Generator ---------------------------------------------------------------------------- */
/* Generator::Generator(RenderDevice*, FFTCalculator*) — src/Generator.cpp:14-27, batched over
 * `cascades` independent cascades (1..OCEAN_MAX_CASCADES) that share the plan's size N. Allocates
 * per cascade: initialSpectrum, heightMap, displacementMap (RGBA32F N*N) and jacobian (R32F N*N)
 * (src/Generator.cpp:99-133). Settings start at the defaults; the first calculate() seeds h0. */
int ocean_generator_create(ocean_generator** out, ocean_fft* fft, int cascades);
/* Generator::~Generator — src/Generator.cpp:29-43 (also frees the jacobian the reference leaks). */
int ocean_generator_destroy(ocean_generator* gen);
int ocean_generator_cascades(const ocean_generator* gen);
/* Generator::GetOceanSettings — src/Generator.h:41. Host-side, mutable; read at calculate(). */
ocean_settings* ocean_generator_settings(ocean_generator* gen, int cascade);
/* Generator::CalculateOcean(float timestep, bool updateOcean) — src/Generator.cpp:45-83, for all
 * cascades: time += timestep (fp32); regenerate h0 when update_spectrum != 0 or on first use;
 * evolve + pack + two EncodeIFFTs + foam. Two fused launches: column pass (evolve + y iFFT of
 * both packed maps) and row pass (x iFFT + row-major maps + Jacobian). */
int ocean_generator_calculate(ocean_generator* gen, float timestep, int update_spectrum);
/* Generator::GenerateSpectrum — src/Generator.cpp:148-154 (the generateSpectrum dispatch). */
int ocean_generator_generate_spectrum(ocean_generator* gen);
/* Getters — src/Generator.h:48-50. Device pointers; heightMap = (h, dh/dx, dh/dz, Dx),
 * displacementMap = (Dz, dDx/dx, dDz/dz, dDx/dz) (src/Generator.h:76-80), jacobian = R32F. */
float* ocean_generator_height_map(ocean_generator* gen, int cascade);
float* ocean_generator_displacement_map(ocean_generator* gen, int cascade);
float* ocean_generator_jacobian_map(ocean_generator* gen, int cascade);
/* The initialSpectrum image (private in the reference, src/Generator.h:86): (h0(k), conj(h0(-k)))
 * per texel, stored strip-blocked: texel (x, y) at index ((x / B) * N + y) * B + (x % B) with
 * B = ocean_generator_spectrum_block(gen), so the column pass streams it contiguously. Slab
 * generators hold only their own columns: the column slab (full spectrum), their kept strips in
 * order, each N * B texels (strip-dealt half spectrum; the Nyquist strip x = 0 .. B-1 last), or their
 * kept columns x = N/2 + u0 .. blocked 64 wide from u0, the last rank then the block of x = 0 .. 63
 * (four-step, ocean_slab_layout half == 2). The pointer is writable: see ocean_generator_set_h0_memo. */
float* ocean_generator_initial_spectrum(ocean_generator* gen, int cascade);
int ocean_generator_spectrum_block(const ocean_generator* gen);

/* Frame path. Half spectrum (default for N = 1024 .. 16384): the column pass transforms only the
 * u >= 0 half of the columns, as 5 complex fields (H, kz H, H/|k|, kz H/|k|, kz^2 H/|k|), and the
 * row pass rebuilds the reference's 4 packed lanes from Hermitian symmetry plus the reference's
 * Nyquist-row term. Whole grids of 1024 .. 4096 use the blocked layout (84 HBM bytes
 * per point instead of 116). N = 8192 / 16384 (whole grids and slabs) run the four-step column pass,
 * whose second step writes destination-block order, so the row pass reads the exchanged blocks
 * directly (124 bytes per point; exchange 20 bytes per point instead of 32); slabs of 1024 .. 4096
 * deal the kept strips over the ranks and move the received fields to row-major before the row pass.
 * enable = 0 selects the full-spectrum path (both give the reference's results within rounding). On a
 * slab generator the switch changes ocean_generator_exchange_bytes and re-seeds h0 at the next frame. */
int ocean_generator_set_half_spectrum(ocean_generator* gen, int enable);
/* N = 8192 / 16384, half spectrum (whole grids and slabs): enable (default) = the column pass in four
 * steps (N = 16 * N2: a 16-point step in registers, then N2-point transforms on 8-column strips
 * written straight into destination-block order; no one-column work items and no transposes; h0 is
 * then blocked ocean_generator_spectrum_block = 64 columns wide, a slab holding only its own kept
 * columns); 0 = the strip-dealt column pass + transposes into row-major fields. Both give the
 * reference's results within rounding. Switching changes ocean_generator_exchange_bytes and re-lays h0
 * out at the next frame from the settings it was seeded with. No reference counterpart. */
int ocean_generator_set_four_step(ocean_generator* gen, int enable);
/* A re-seed requested by ocean_generator_calculate(.., update_spectrum = 1) — the reference app
 * requests one on every frame (src/Waves.cpp:91-94) — is skipped when no h0 input (every settings
 * field but `time`) changed since h0 was last seeded: it would reproduce the same image bit for bit.
 * Handing out the h0 pointer (ocean_generator_initial_spectrum) makes the next requested re-seed run,
 * since the caller may have written h0 through it. enable = 0 re-seeds on every request, as the
 * reference does. Default 1. No reference counterpart. */
int ocean_generator_set_h0_memo(ocean_generator* gen, int enable);
/* Frame overlap (whole grids of N = 1024 .. 4096 on the half-spectrum path): frame f + 1's column
 * pass, which depends only on h0 and the time, runs on an internal stream into a second set of field
 * buffers while frame f's row pass still runs on the generator's stream, so the two passes' launch
 * tails overlap when the caller issues frames back to back. Row passes, maps and Jacobian stay in
 * order on the generator's stream, and the results are bit-identical. The internal stream waits for
 * the generator's stream whenever the library writes h0 (seeding, re-seeds) and after the h0 pointer
 * is handed out (ocean_generator_initial_spectrum); other work the caller enqueues on that stream
 * between frames is not waited for, so it must not write the generator's buffers. Costs 20 B of
 * device memory per point. Pays at 1-2 cascades per generator of 1024^2 (8 x 4096^2: slower, leave it
 * off). At 2048 and 4096 with 1-2 cascades the column pass runs on half strips, which share CUs with
 * the overlapped row pass: there the serial frame is faster (0.318 against 0.346 ms at one cascade of
 * 4096, profiles/r04_halfbench_xgrid_fb2_1.log; 0.087 against 0.091 ms at one of 2048,
 * profiles/r06g_configs.md), so leave it off as well.
 * Default 0. No reference counterpart (the reference barriers after every dispatch). */
int ocean_generator_set_frame_overlap(ocean_generator* gen, int enable);
/* Algorithmic HBM bytes per height-field point of the column pass [0] and the row pass [1] of the
 * generator's current path (what bench.py prices the roofline with). */
int ocean_generator_frame_bytes(const ocean_generator* gen, double per_point[2]);

/* ---- slab decomposition of one grid over several GPUs ------------------------------------- */
/* One N x N cascade split over `ranks` GPUs (power of two <= 16), this process being `rank`: the
 * column pass works on columns [rank*w, rank*w + w), the row pass on rows [rank*w, rank*w + w),
 * w = N / ranks (the reference runs everything on one device). With the half spectrum
 * (default for N >= 1024) the column pass works on the rank's share of the kept strips instead of
 * the column slab. A frame is:
 *   ocean_generator_slab_columns(gen, dt, update, send)  time += dt, h0 if needed, evolve + y iFFT
 *   all-to-all with equal splits of ocean_generator_exchange_bytes(gen) / ranks bytes: the block at
 *     send + q * bytes/ranks goes to rank q and arrives at recv + rank_src * bytes/ranks (RCCL)
 *   ocean_generator_slab_rows(gen, recv)                 x iFFT + maps + Jacobian of the row slab
 * send/recv are caller-owned device buffers (null = the generator's internal buffer, which is what
 * ranks == 1 uses). The map getters then address the row slab: w rows x N texels, row-major. */
int ocean_generator_create_slab(ocean_generator** out, ocean_fft* fft, int rank, int ranks);
size_t ocean_generator_exchange_bytes(const ocean_generator* gen);
int ocean_generator_slab_columns(ocean_generator* gen, float timestep, int update_spectrum, float* send);
int ocean_generator_slab_rows(ocean_generator* gen, const float* recv);
int ocean_generator_slab_info(const ocean_generator* gen, int* rank, int* ranks, int* row0, int* rows);
/* Host-only geometry of a one-cascade slab generator (no device needed): out = {first kept strip,
 * strips this rank transforms, strip slots per block, rows per block (N / ranks), exchange block
 * bytes, exchange bytes} for the strip-dealt half-spectrum path (half == 1: the STRIPS = N / (2B) + 1
 * kept strips dealt ceil(STRIPS / ranks) per rank); {first kept column u0, kept columns N / (2 ranks),
 * 1 if the rank also holds the Nyquist column, rows, block bytes, exchange bytes} for the four-step
 * path (half == 2, N = 8192 / 16384: the default there); or {first column, columns, 0, rows, block
 * bytes, exchange bytes} for the full-spectrum path (half == 0). */
int ocean_slab_layout(size_t texture_size, int rank, int ranks, int half, int64_t out[6]);

/* ---- the slab exchange over RCCL (xGMI) ---------------------------------------------------
 * The frame of a slab generator with the all-to-all inside the library: P grouped ncclSend /
 * ncclRecv pairs of exchange_bytes / P between the column and the row pass, on the
 * generator's stream (serial) or on a second stream (pipelined). The communicator spans the P ranks
 * of the grid, rank r = the slab rank (one process per GPU, the current HIP device). */
#define OCEAN_COMM_ID_BYTES 128
typedef struct ocean_comm ocean_comm;
/* ncclGetUniqueId: created by one rank and handed to every rank's ocean_comm_create by the caller
 * (MPI, a file, torch.distributed ...). */
int ocean_comm_unique_id(unsigned char id[OCEAN_COMM_ID_BYTES]);
/* ncclCommInitRank(nranks, id, rank) on the current device; collective over the nranks processes. */
int ocean_comm_create(ocean_comm** out, const unsigned char id[OCEAN_COMM_ID_BYTES], int nranks, int rank);
/* Use a communicator the caller already has (an ncclComm_t; not destroyed by ocean_comm_destroy).
 * nranks / rank must be the communicator's own (ncclCommCount / ncclCommUserRank), else
 * OCEAN_ERR_INVALID. A communicator must outlive every generator whose frames used it: destroying
 * a generator drains its exchange stream but does not issue a pending pipelined frame's row pass. */
int ocean_comm_wrap(ocean_comm** out, void* nccl_comm, int nranks, int rank);
int ocean_comm_destroy(ocean_comm* comm);
/* The equal-split all-to-all of caller device buffers over the communicator (bytes / nranks to each
 * rank), enqueued on hip_stream: for callers that run ocean_generator_slab_columns / _rows themselves. */
int ocean_comm_all_to_all(ocean_comm* comm, const void* send, void* recv, size_t bytes, void* hip_stream);
/* One frame: time += dt, h0 if needed, column pass into the library's send buffer, the all-to-all,
 * row pass — all enqueued on the generator's stream (src/Generator.cpp:45-83 over P ranks). */
int ocean_generator_slab_frame(ocean_generator* gen, ocean_comm* comm, float timestep, int update_spectrum);
/* Pipelined frames over two buffer slots: frame f's all-to-all runs on a second stream beside frame
 * f + 1's column pass and frame f - 1's row pass, so the steady state is max(exchange, passes); the
 * maps lag the last issued frame by one until ocean_generator_slab_flush. Size the passes with
 * ocean_fft_set_cu_budget to leave CUs to RCCL's kernels. */
int ocean_generator_slab_frame_pipelined(ocean_generator* gen, ocean_comm* comm, float timestep, int update_spectrum);
int ocean_generator_slab_flush(ocean_generator* gen);

/* ---- the one-sided slab exchange over peer-mapped memory (IPC, xGMI) -----------------------
 * No send buffer and no copy kernel: the column pass's second step stores block q of its output
 * straight into rank q's receive slot, through a mapping of rank q's device memory (hipIpc handles
 * exchanged by the caller), and the row pass reads its own slot. Per frame each rank raises one
 * flag word in every rank's flag array after its stores ("ready") and one after its row pass has
 * read its slot ("freed"); the waits for them are small kernels on the streams (one wave per workgroup,
 * dealt over every XCD, each ending in a system-scope acquire), bounded by a
 * timeout (ocean_peers_set_timeout), so a missing peer never holds the GPU: the frame goes on, and
 * ocean_peers_synchronize reports OCEAN_ERR_TIMEOUT. Every half-spectrum slab path (N >= 1024): on the
 * four-step slabs (N = 8192 / 16384) step 2 puts, on the strip-dealt ones the column pass itself; the
 * RCCL exchange above also serves the full-spectrum slabs below 1024. SURVEY §8e, the reference's
 * CalculateOcean (src/Generator.cpp:45-83) split over P ranks.
 * Use: ocean_peers_create on every rank, ocean_peers_handle -> the caller gathers the P handles (in
 * rank order, e.g. an all-gather) -> ocean_peers_connect; frames; ocean_peers_synchronize on every
 * rank and a host barrier across ranks before ocean_peers_destroy (a peer may still signal). */
#define OCEAN_ERR_TIMEOUT 5   /* a peer's frame signal did not arrive within the timeout */
#define OCEAN_PEER_HANDLE_BYTES 256
typedef struct ocean_peers ocean_peers;
/* Two receive slots of ocean_generator_exchange_bytes(gen) and the flag words, in this process's
 * device memory; gen must be a slab generator on a half-spectrum path (N >= 1024). A later path switch
 * that changes the exchange size makes the peers refuse frames. */
int ocean_peers_create(ocean_peers** out, ocean_generator* gen);
int ocean_peers_destroy(ocean_peers* peers);
/* This rank's handle (rank, ranks, slot size, the IPC handles of its slots and flags). */
int ocean_peers_handle(const ocean_peers* peers, unsigned char handle[OCEAN_PEER_HANDLE_BYTES]);
/* Map every other rank's slots and flags: handles = ranks * OCEAN_PEER_HANDLE_BYTES, in rank order
 * (this rank's own entry is checked and used locally). */
int ocean_peers_connect(ocean_peers* peers, const unsigned char* handles);
/* The same for `ranks` ocean_peers of one process on one device (the single-GPU emulation of a P-rank
 * grid, tests): each rank's peers are the others' buffers directly, no IPC. */
int ocean_peers_connect_local(ocean_peers* const* all, int ranks);
/* Wait timeout in milliseconds (default 20000). */
int ocean_peers_set_timeout(ocean_peers* peers, int ms);
/* CUs the put kernels (the Nyquist-row term and step 2) are sized for (0 = the plan's budget): with
 * the stores bound by xGMI, fewer workgroups leave the other CUs to the row pass of the previous
 * frame in the pipelined frame. */
int ocean_peers_set_put_cus(ocean_peers* peers, int cus);
/* The streams pipelined frames run step 1 of the column pass, the put and the row pass on (null: the
 * peers' own; the generator's stream waits for each row pass, so the maps stay ordered on it). The
 * one-GPU emulation gives all P ranks one set, as one GPU has one path out over xGMI. */
int ocean_peers_set_streams(ocean_peers* peers, void* column_stream, void* put_stream, void* row_stream);
/* The CUs the caller's row stream may use when it is CU-masked (0 = all, the default; the peers' own
 * masked streams know theirs): the 16384 row pass loops over rows on a resident grid, one workgroup per
 * CU, so a grid sized for CUs the stream cannot use leaves whole workgroups waiting for a second turn. */
int ocean_peers_set_row_cus(ocean_peers* peers, int cus);
/* Recreate the peers' own streams CU-masked: the put on `cus_per_xcd` CUs of every XCD, step 1 and the
 * row pass on the others (0: unmasked, the default). An xGMI-bound put then holds only its own CUs
 * while it waits on the links. (A CU mask splits every XCD alike: workgroups are dealt to all 8 XCDs
 * whatever the mask, and an XCD left without mask bits runs on all its CUs.) */
int ocean_peers_set_put_cu_mask(ocean_peers* peers, int cus_per_xcd);
/* Serial frame on the generator's stream: time += dt, h0 if needed, step 1, wait for the slot, put,
 * signal; wait for every rank's blocks, row pass, signal. */
int ocean_generator_slab_frame_put(ocean_generator* gen, ocean_peers* peers, float timestep, int update_spectrum);
/* Pipelined: frame f's step 1 on the peers' column stream (into one of two parts slots), its put on
 * their put stream, beside frame f + 1's step 1 and frame f - 1's row pass on the generator's stream
 * (two receive slots); the maps lag by one frame until ocean_peers_flush. */
int ocean_generator_slab_frame_put_pipelined(ocean_generator* gen, ocean_peers* peers, float timestep,
                                             int update_spectrum);
int ocean_peers_flush(ocean_peers* peers);
/* The two halves of a serial frame, for callers (and the one-GPU emulation) that issue the column
 * passes of all ranks before their row passes: columns + put + signal; wait + rows + signal. */
int ocean_generator_slab_put_columns(ocean_generator* gen, ocean_peers* peers, float timestep, int update_spectrum);
int ocean_generator_slab_put_rows(ocean_generator* gen, ocean_peers* peers);
/* Wait for this rank's streams; OCEAN_ERR_TIMEOUT when any wait gave up (which, and at which frame,
 * in ocean_last_error). After a timeout the device-side error word is cleared and the peers refuse every
 * further frame with OCEAN_ERR_TIMEOUT (the ranks' flag counts no longer agree): destroy and recreate
 * them. Pipelined row passes wait for the caller's work on the generator's stream before they rewrite
 * the maps, and h0 re-seeds wait for the column pass still reading h0 on the peers' streams. */
int ocean_peers_synchronize(ocean_peers* peers);

/* Receive slot `slot` (0 or 1) of this rank: its device pointer and size (frame f's blocks land in
 * slot f % 2). Debug only (tests/test_gpu_peers.py reads a slot into every XCD's L2 just before the
 * peers' put rewrites it, to check that the row pass never reads a stale line). No reference counterpart. */
int ocean_peers_debug_slot(const ocean_peers* peers, int slot, void** ptr, size_t* bytes);

/* The whole-grid half-spectrum frame's layout pairing (N = 1024 .. 4096), host only: out = the field
 * strip width, gab/gde row group, gc row group and h0 strip width the column pass WRITES / reads {0..3},
 * the first three as the row pass (rows_variant 1 = k_rows_hp at 4096, 0 = k_rows_half) READS them
 * {4..6}, and the h0 strip width the seeding writes {7}. Each launcher picks its kernel from the same
 * descriptor it reports here (tests/test_capi_cpu.py checks the pairs over every shape). */
int ocean_frame_plan(size_t texture_size, int cascades, int rows_variant, int32_t out[8]);

/* ---- instrumentation (bench) ------------------------------------------------------------- */
/* When enabled, each kernel launch of the generator is bracketed by HIP events on its stream. */
int ocean_generator_set_profiling(ocean_generator* gen, int enable);
/* Synchronises, then returns per-kernel totals since the last call and resets them.
 * Index 0 = spectrum (h0), 1 = column pass (evolve + y iFFT), 2 = row pass (x iFFT + foam). */
int ocean_generator_kernel_times(ocean_generator* gen, double ms_total[3], int64_t launches[3]);
/* The same with index 3 = the put of one-sided frames (the slot wait + the Nyquist-row term + step 2).
 * Index 1 includes it in serial frames; in pipelined ones index 1 is step 1 alone (its own stream). */
int ocean_generator_kernel_times4(ocean_generator* gen, double ms_total[4], int64_t launches[4]);

/* ---- debug -------------------------------------------------------------------------------- */
/* Device Hash (resources/spectrum.compute:109-117) of count (x, y) pairs in device memory:
 * raw[i] = uint32 n, uv[2i..2i+1] = the two uniforms. For bit-exact parity tests. */
int ocean_debug_hash(const uint32_t* xy, int count, uint32_t* raw, float* uv, void* hip_stream);
/* Copy `bytes` (a multiple of 16, 16-B aligned device pointers) with exactly `workgroups` 256-thread
 * workgroups on hip_stream: a rate-limited HBM read + write stream (bench.py prices a slab rank's
 * exchange traffic with it on one GPU). No reference counterpart. */
int ocean_debug_copy(void* dst, const void* src, size_t bytes, int workgroups, void* hip_stream);

/* ---- Surface consumer: the renderer's use of the maps -------------------
 * resources/waveShader.glsl evaluated per mesh vertex on the maps of `count` (generator, cascade)
 * pairs (the reference binds 3 generators, src/Renderer.cpp:62-72; here 1..16, one map size,
 * whole-grid generators): the vertex stage's displacement loop (:101-110; cascade i samples at the
 * position cascades < i displaced), then at the displaced position the fragment stage's slope
 * normal and Jacobian average (:127-144). Sampling is GL_LINEAR + GL_REPEAT in fp32
 * (src/Generator.cpp:116-119). Output per vertex: 8 floats (x, y, z, jacobian, nx, ny, nz, 0),
 * device memory, written on the first generator's stream. planeSize / displacement come from each
 * cascade's settings (Renderer.cpp:70-71). A request of at least 65536 vertices and 4 per map
 * texel first repacks the channels each stage reads into an atlas (2 x 16 B per texel and cascade,
 * at most 256 MiB, owned by the first generator's FFT plan and kept for later requests), then samples
 * it: the same bits, fewer load instructions. No reference counterpart as a call: it replaces the
 * vertex + fragment shader sampling. */
int ocean_surface_sample(ocean_generator* const* gens, const int* cascades, int count, const float* xz,
                         int64_t points, float* out);
/* The same on the reference's plane mesh (40 m x 40 m, res x res quads, (res+1)^2 vertices, x
 * fastest; src/Renderer.cpp:18) through the camera-relative warp of waveShader.glsl:77-98:
 * camera = {viewInverse[3].x, .y, .z, forward.x, forward.z} with forward = -viewInverse[0]. */
int ocean_surface_sample_plane(ocean_generator* const* gens, const int* cascades, int count, const float camera[5],
                               int res, float* out);

#ifdef __cplusplus
}
#endif

#endif /* OCEANFFT_H */
