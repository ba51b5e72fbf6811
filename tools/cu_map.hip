// cu_map.hip - which CUs (XCD, shader engine, CU) a stream's CU mask (hipExtStreamCreateWithCUMask)
// lets a kernel use on this device.  For each test mask a stream runs 4,096 one-wave workgroups
// that each hold their CU for ~20 us and record their XCC_ID and HW_ID registers; the tool prints,
// per mask, how many distinct CUs each XCD served and which (se, cu) those were.
//   hipcc --offload-arch=gfx950 -O2 tools/cu_map.hip -o tools/cu_map && tools/cu_map
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <set>
#include <string>
#include <vector>

__global__ void where(unsigned *out) {
  // HW_REG_XCC_ID (20): bits [3:0] = XCC; HW_REG_HW_ID (4): CU_ID [11:8], SH_ID [12], SE_ID [15:13]
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(2);  // ~20 us at 100 MHz
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
}

int main() {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
  const int ncu = prop.multiProcessorCount, nb = 4096;
  unsigned *d = nullptr;
  if (hipMalloc(&d, 2 * nb * sizeof(unsigned)) != hipSuccess) return 1;
  std::vector<unsigned> h(2 * nb);
  printf("# %d CUs\n", ncu);
  struct T { const char *name; bool (*in)(int); };
  const T tests[] = {
      {"all", [](int) { return true; }},
      {"bits 0-127", [](int b) { return b < 128; }},
      {"bits 128-255", [](int b) { return b >= 128; }},
      {"bits 0-31", [](int b) { return b < 32; }},
      {"b%8==0", [](int b) { return b % 8 == 0; }},
      {"b%8!=0", [](int b) { return b % 8 != 0; }},
      {"b<224", [](int b) { return b < 224; }},
      {"b>=224", [](int b) { return b >= 224; }},
      {"b%32<28", [](int b) { return b % 32 < 28; }},
      {"b%32>=28", [](int b) { return b % 32 >= 28; }},
  };
  for (const T &t : tests) {
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    for (int b = 0; b < ncu; b++)
      if (t.in(b)) mask[b / 32] |= 1u << (b % 32);
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) return 2;
    hipMemsetAsync(d, 0xff, 2 * nb * sizeof(unsigned), s);
    where<<<nb, 64, 0, s>>>(d);
    if (hipStreamSynchronize(s) != hipSuccess) return 3;
    hipMemcpy(h.data(), d, 2 * nb * sizeof(unsigned), hipMemcpyDeviceToHost);
    std::set<unsigned> cus[16];
    for (int i = 0; i < nb; i++) cus[h[2 * i] & 15u].insert(((h[2 * i + 1] >> 13) & 7u) * 16 + ((h[2 * i + 1] >> 8) & 15u));
    printf("%-14s", t.name);
    int tot = 0;
    for (int x = 0; x < 8; x++) {
      printf(" x%d:%zu", x, cus[x].size());
      tot += (int)cus[x].size();
    }
    printf("  total %d\n", tot);
    for (int x = 0; x < 8; x++) {
      std::string l;
      for (unsigned c : cus[x]) l += " " + std::to_string(c >> 4) + "." + std::to_string(c & 15);
      printf("    x%d:%s\n", x, l.c_str());
    }
    hipStreamDestroy(s);
  }
  hipFree(d);
  return 0;
}
