// xcdprobe.hip — raw HW_REG_XCC_ID / HW_REG_HW_ID of the workgroups of CU-masked streams (a few
// single-CU masks and no mask), to read how hipExtStreamCreateWithCUMask bits map onto XCDs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

__global__ void k_ids(unsigned* out)
{
  if (threadIdx.x == 0)
  {
    out[2 * blockIdx.x] = __builtin_amdgcn_s_getreg((31 << 11) | 20);     // HW_REG_XCC_ID, all bits
    out[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_HW_ID, all bits
  }
}

int main()
{
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = 1024;
  unsigned* d = nullptr;
  (void)hipMalloc(&d, 2 * blocks * sizeof(unsigned));
  std::vector<unsigned> h(2 * blocks);
  // masks: -1 none; 0..255 one CU; 1000 = bits 0..31; 1001 = c % 32 < 4; 1002 = c % 8 >= 6; 1003 = c < 64
  std::vector<int> probe = {-1, 0, 33, 1000, 1001, 1002, 1003};
  for (int c : probe)
  {
    hipStream_t s;
    if (c < 0)
      (void)hipStreamCreate(&s);
    else
    {
      std::vector<uint32_t> mask((cus + 31) / 32, 0u);
      for (int k = 0; k < cus; k++)
      {
        const bool in = c < 1000 ? k == c : c == 1000 ? k < 32 : c == 1001 ? k % 32 < 4 : c == 1002 ? k % 8 >= 6 : k < 64;
        if (in)
          mask[k / 32] |= 1u << (k % 32);
      }
      (void)hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
    }
    hipLaunchKernelGGL(k_ids, dim3(blocks), dim3(64), 0, s, d);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
    std::map<unsigned, int> xcc, cu;
    for (int b = 0; b < blocks; b++)
    {
      xcc[h[2 * b]]++;
      const unsigned hw = h[2 * b + 1];
      cu[(h[2 * b] & 0xF) << 16 | ((hw >> 8) & 0xF) | ((hw >> 13) & 0x3) << 4 | ((hw >> 12) & 1) << 6]++;
    }
    std::printf("mask %s%d: XCC_ID raw values {", c < 0 ? "none " : "cu ", c);
    for (auto& kv : xcc)
      std::printf(" 0x%x:%d", kv.first, kv.second);
    std::printf(" }, distinct (xcc, se, sh, cu) = %zu; first blocks:", cu.size());
    for (int b = 0; b < 10; b++)
      std::printf(" [x%u hw%08x]", h[2 * b] & 0xF, h[2 * b + 1]);
    std::printf("\n");
    (void)hipStreamDestroy(s);
  }
  return 0;
}
