// device/memory.h — global-memory access: buffer (SRD) loads/stores with cache-policy bits, and the
// opaque() register-pressure guard.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>


namespace oceanfft
{

// ------------------------------------------------------------------------------------------------
// Buffer (SRD) global access: wave-uniform base in SGPRs + one 32-bit lane offset (T8 in the CDNA
// guide). Keeps the 16 per-thread element addresses out of VGPRs. Offsets stay < 2^31 bytes.
// ------------------------------------------------------------------------------------------------
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t srd(const void* base, int num_bytes)
{
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, num_bytes, 0x00020000);
}

// Raw-buffer range checking: a load at or past num_bytes returns 0 and a store there is dropped,
// which handles ragged row blocks without branches.
constexpr int kAllBytes = 0x7FFFFFFF;

// AUX: cache-policy bits of the buffer instruction (0 = default; 2 = nt, streaming / non-temporal).
template <int AUX = 0>
__device__ __forceinline__ float4 ld4(const void* base, int voff_bytes, int num_bytes = kAllBytes)
{
  f4v r = __builtin_amdgcn_raw_buffer_load_b128(srd(base, num_bytes), voff_bytes, 0, AUX);
  return make_float4(r.x, r.y, r.z, r.w);
}

template <int AUX = 0>
__device__ __forceinline__ void st4(void* base, int voff_bytes, float4 v, int num_bytes = kAllBytes)
{
  f4v r = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(r, srd(base, num_bytes), voff_bytes, 0, AUX);
}

typedef unsigned int u2v __attribute__((ext_vector_type(2)));

template <int AUX = 0>
__device__ __forceinline__ float2 ld2(const void* base, int voff_bytes)
{
  u2v r = __builtin_amdgcn_raw_buffer_load_b64(srd(base, kAllBytes), voff_bytes, 0, AUX);
  return make_float2(__uint_as_float(r.x), __uint_as_float(r.y));
}

template <int AUX = 0>
__device__ __forceinline__ void st2(void* base, int voff_bytes, float2 v)
{
  u2v r = {__float_as_uint(v.x), __float_as_uint(v.y)};
  __builtin_amdgcn_raw_buffer_store_b64(r, srd(base, kAllBytes), voff_bytes, 0, AUX);
}

template <int AUX = 0>
__device__ __forceinline__ void st1(void* base, int voff_bytes, float v)
{
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), srd(base, kAllBytes), voff_bytes, 0, AUX);
}

// The same with a second, wave-uniform byte offset (the piece offset m * stride of a call site that
// touches 16 pieces of one buffer per item): ONE descriptor (4 SGPRs) per buffer, the piece offset
// added to the lane offset in the VGPR voffset. k_cols_half built one descriptor per piece (~50 per
// item) and spilled SGPRs to VGPR lanes (476 v_readlane/v_writelane per item at 112 SGPRs).
// OCEAN_SOFFSET_PIECES (tools/microbench/detbench only) passes the piece offset in the instruction's
// SGPR soffset field instead: the build round 2 recorded as non-deterministic.
#if defined(OCEAN_SOFFSET_PIECES)
#define OCEAN_PIECE(voff, soff) (voff), (soff)
#else
#define OCEAN_PIECE(voff, soff) (voff) + (soff), 0
#endif
template <int AUX = 0>
__device__ __forceinline__ float4 ld4s(const void* base, int voff_bytes, int soff_bytes)
{
  f4v r = __builtin_amdgcn_raw_buffer_load_b128(srd(base, kAllBytes), OCEAN_PIECE(voff_bytes, soff_bytes), AUX);
  return make_float4(r.x, r.y, r.z, r.w);
}

template <int AUX = 0>
__device__ __forceinline__ void st4s(void* base, int voff_bytes, int soff_bytes, float4 v)
{
  f4v r = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(r, srd(base, kAllBytes), OCEAN_PIECE(voff_bytes, soff_bytes), AUX);
}

template <int AUX = 0>
__device__ __forceinline__ float2 ld2s(const void* base, int voff_bytes, int soff_bytes)
{
  u2v r = __builtin_amdgcn_raw_buffer_load_b64(srd(base, kAllBytes), OCEAN_PIECE(voff_bytes, soff_bytes), AUX);
  return make_float2(__uint_as_float(r.x), __uint_as_float(r.y));
}

template <int AUX = 0>
__device__ __forceinline__ void st2s(void* base, int voff_bytes, int soff_bytes, float2 v)
{
  u2v r = {__float_as_uint(v.x), __float_as_uint(v.y)};
  __builtin_amdgcn_raw_buffer_store_b64(r, srd(base, kAllBytes), OCEAN_PIECE(voff_bytes, soff_bytes), AUX);
}

__device__ __forceinline__ int clamp_bytes(int64_t b)
{
  return b > kAllBytes ? kAllBytes : (b < 0 ? 0 : (int)b);
}


// Hide a loop-invariant value from LICM: without this, hipcc hoists ~100 per-thread LDS/global
// address computations out of the persistent loops and spills them to scratch.
__device__ __forceinline__ int opaque(int v)
{
  asm volatile("" : "+v"(v));
  return v;
}

// The same for a wave-uniform 64-bit value kept in SGPRs: computed where it is used, not hoisted.
__device__ __forceinline__ size_t sopaque(size_t v)
{
  asm volatile("" : "+s"(v));
  return v;
}

__device__ __forceinline__ int sopaque(int v)
{
  asm volatile("" : "+s"(v));
  return v;
}

}  // namespace oceanfft
