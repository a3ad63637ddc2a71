// xcdmask.hip — the XCD of every logical CU index of hipExtStreamCreateWithCUMask (ocean_peers_set_put_xcds
// masks whole XCDs). For each CU c, 64 one-wave workgroups on a stream masked to {c} record
// HW_REG_XCC_ID; prints c -> XCD for all CUs, whether each CU kept its workgroups on one XCD, and which
// simple rule (c / (CUs/8), or c % 8) the map follows. Exit 0 when every CU maps to one XCD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <vector>

#define CHECK(x)                                                                  \
  do                                                                              \
  {                                                                               \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess)                                                         \
    {                                                                             \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                         \
      return 2;                                                                   \
    }                                                                             \
  } while (0)

__global__ void k_xcc(unsigned* out)
{
  if (threadIdx.x == 0)
    out[blockIdx.x] = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xF;  // HW_REG_XCC_ID[3:0]
}

int main()
{
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = 64;
  unsigned* d = nullptr;
  CHECK(hipMalloc(&d, blocks * sizeof(unsigned)));
  std::vector<unsigned> h(blocks);
  std::vector<int> xcd(cus, -1);
  bool one = true;
  for (int c = 0; c < cus; c++)
  {
    std::vector<uint32_t> mask((cus + 31) / 32, 0u);
    mask[c / 32] |= 1u << (c % 32);
    hipStream_t s;
    CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    hipLaunchKernelGGL(k_xcc, dim3(blocks), dim3(64), 0, s, d);
    CHECK(hipGetLastError());
    CHECK(hipStreamSynchronize(s));
    CHECK(hipMemcpy(h.data(), d, blocks * sizeof(unsigned), hipMemcpyDeviceToHost));
    std::set<int> seen(h.begin(), h.end());
    one = one && seen.size() == 1;
    xcd[c] = seen.size() == 1 ? (int)*seen.begin() : -1;
    CHECK(hipStreamDestroy(s));
  }
  CHECK(hipFree(d));
  std::printf("cu -> xcd:");
  for (int c = 0; c < cus; c++)
    std::printf("%s%d", c % 32 ? " " : "\n  ", xcd[c]);
  std::printf("\n");
  bool div = true, mod = true;
  std::vector<std::set<int>> by_div(8), by_mod(8);
  for (int c = 0; c < cus; c++)
  {
    by_div[c / (cus / 8)].insert(xcd[c]);
    by_mod[c % 8].insert(xcd[c]);
  }
  for (int k = 0; k < 8; k++)
  {
    div = div && by_div[k].size() == 1;
    mod = mod && by_mod[k].size() == 1;
  }
  std::printf("every CU on one XCD: %s; rule c / %d: %s; rule c %% 8: %s\n", one ? "yes" : "no", cus / 8,
              div ? "yes" : "no", mod ? "yes" : "no");
  return one ? 0 : 1;
}
