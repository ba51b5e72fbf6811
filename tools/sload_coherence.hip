// sload_coherence.hip - does a scalar load with glc see another workgroup's vector stores while a
// kernel runs?  Workgroup 0 stores 1..N into a word (one store every ~1 us); every other workgroup
// polls the word with `s_load_dword ... glc` (and, for comparison, a relaxed agent-scope vector
// atomic load) and records how many distinct values each form saw.  Workgroups 8 apart share an
// XCD (round-robin dispatch), others do not.
//   hipcc --offload-arch=gfx950 -O2 tools/sload_coherence.hip -o tools/sload_coherence
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned *word, unsigned *out, int n) {
  const int wg = blockIdx.x;
  if (wg == 0) {
    for (int i = 1; i <= n; i++) {
      if (threadIdx.x == 0) asm volatile("global_store_dword %0, %1, off" ::"v"(word), "v"((unsigned)i) : "memory");
      const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
      while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < 100) __builtin_amdgcn_s_sleep(2);
    }
    return;
  }
  unsigned last_s = 0, seen_s = 0, last_v = 0, seen_v = 0;
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < 100LL * (n + 20)) {
    unsigned v;
    asm volatile("s_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(word) : "memory");
    if (v != last_s) { seen_s++; last_s = v; }
    const unsigned u = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (u != last_v) { seen_v++; last_v = u; }
    __builtin_amdgcn_s_sleep(4);
  }
  if (threadIdx.x == 0) {
    out[4 * wg] = seen_s;
    out[4 * wg + 1] = last_s;
    out[4 * wg + 2] = seen_v;
    out[4 * wg + 3] = last_v;
  }
}

int main() {
  const int nwg = 24, n = 200;
  unsigned *word, *out;
  hipMalloc(&word, 256);
  hipMalloc(&out, 4 * nwg * 4);
  hipMemset(word, 0, 256);
  hipMemset(out, 0, 4 * nwg * 4);
  probe<<<nwg, 64>>>(word, out, n);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  unsigned h[4 * nwg];
  hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
  printf("writer: workgroup 0, values 1..%d\n# wg  same_xcd  s_load_glc: distinct last   vector_atomic: distinct last\n", n);
  for (int w = 1; w < nwg; w++)
    printf("%3d %d %6u %6u   %6u %6u\n", w, w % 8 == 0, h[4 * w], h[4 * w + 1], h[4 * w + 2], h[4 * w + 3]);
  return 0;
}
