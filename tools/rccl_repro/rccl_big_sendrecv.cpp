// Standalone RCCL check, no oceanfft code: one rank (world size 1), one ncclSend / ncclRecv self pair
// of `MiB` bytes (ncclUint8) in one group on one stream, as ocean_comm_all_to_all issued it before the
// 512-MiB pieces (profiles/r03_rccl_selfcheck.log: wrong from 1400 MiB through the library). If this
// program reproduces the corruption, the fault is RCCL's; if not, it was the library's byte arithmetic.
// Usage: rccl_big_sendrecv [MiB ...]   (default 1 64 512 1024 1400 2100 3000)
// Build: tools/rccl_repro/Makefile (one binary against /opt/rocm's librccl, one against torch's).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK_HIP(x)                                                                               \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      return 2;                                                                                    \
    }                                                                                              \
  } while (0)
#define CHECK_NCCL(x)                                                                              \
  do {                                                                                             \
    ncclResult_t r_ = (x);                                                                         \
    if (r_ != ncclSuccess) {                                                                       \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(r_));      \
      return 2;                                                                                    \
    }                                                                                              \
  } while (0)

// byte i of the pattern: a hash of i, so a shifted or truncated copy cannot match by accident
__device__ __host__ inline unsigned char pattern(size_t i)
{
  unsigned long long x = (unsigned long long)i * 0x9E3779B97F4A7C15ull;
  x ^= x >> 29;
  return (unsigned char)(x ^ (x >> 8) ^ 0x5Au);
}

__global__ void fill(unsigned char* p, size_t n)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = pattern(i);
}

// counts mismatching bytes and records the first and last mismatching offsets
__global__ void check(const unsigned char* p, size_t n, unsigned long long* out)
{
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (p[i] != pattern(i)) {
      atomicAdd(&out[0], 1ull);
      atomicMin(&out[1], (unsigned long long)i);
      atomicMax(&out[2], (unsigned long long)i);
    }
}

int main(int argc, char** argv)
{
  std::vector<size_t> mibs;
  for (int a = 1; a < argc; a++)
    mibs.push_back(std::strtoull(argv[a], nullptr, 10));
  if (mibs.empty())
    mibs = {1, 64, 512, 1024, 1400, 2100, 3000};
  int version = 0;
  CHECK_NCCL(ncclGetVersion(&version));
  std::printf("RCCL version code %d\n", version);
  ncclUniqueId id;
  CHECK_NCCL(ncclGetUniqueId(&id));
  ncclComm_t comm;
  CHECK_NCCL(ncclCommInitRank(&comm, 1, id, 0));
  hipStream_t s;
  CHECK_HIP(hipStreamCreate(&s));
  unsigned long long* stats;
  CHECK_HIP(hipMalloc(&stats, 3 * sizeof(unsigned long long)));
  int bad = 0;
  for (size_t mib : mibs) {
    const size_t n = mib << 20;
    unsigned char *send = nullptr, *recv = nullptr;
    CHECK_HIP(hipMalloc(&send, n));
    CHECK_HIP(hipMalloc(&recv, n));
    CHECK_HIP(hipMemsetAsync(recv, 0, n, s));
    fill<<<4096, 256, 0, s>>>(send, n);
    CHECK_HIP(hipGetLastError());
    CHECK_NCCL(ncclGroupStart());
    CHECK_NCCL(ncclSend(send, n, ncclUint8, 0, comm, s));
    CHECK_NCCL(ncclRecv(recv, n, ncclUint8, 0, comm, s));
    CHECK_NCCL(ncclGroupEnd());
    const unsigned long long init[3] = {0ull, ~0ull, 0ull};
    CHECK_HIP(hipMemcpyAsync(stats, init, sizeof(init), hipMemcpyHostToDevice, s));
    check<<<4096, 256, 0, s>>>(recv, n, stats);
    CHECK_HIP(hipGetLastError());
    unsigned long long h[3];
    CHECK_HIP(hipMemcpyAsync(h, stats, sizeof(h), hipMemcpyDeviceToHost, s));
    CHECK_HIP(hipStreamSynchronize(s));
    if (h[0] == 0)
      std::printf("%zu MiB (%zu bytes): exact\n", mib, n);
    else {
      bad++;
      std::printf("%zu MiB (%zu bytes): %llu bytes wrong, first at %llu, last at %llu\n", mib, n, h[0], h[1], h[2]);
    }
    std::fflush(stdout);
    CHECK_HIP(hipFree(send));
    CHECK_HIP(hipFree(recv));
  }
  CHECK_NCCL(ncclCommDestroy(comm));
  CHECK_HIP(hipFree(stats));
  CHECK_HIP(hipStreamDestroy(s));
  std::printf("%s\n", bad ? "CORRUPTED" : "ALL EXACT");
  return bad ? 1 : 0;
}
