// gap_micro.hip - the per-step launch floor of the finest level's chain, isolated (VERDICT r4
// item 2): kernel boundaries between a K3p-shaped launch (256 workgroups x 512 threads, 150 KiB
// LDS, one per CU) and a merge-shaped one (342 one-wave workgroups), alternating on one stream,
// launched eagerly or replayed from a captured hipGraph.  Each workgroup stamps its first and
// last s_memrealtime tick; a boundary = the next launch's earliest start - the previous launch's
// latest end (as bench.py's chain_gap_us_timed).
//   hipcc --offload-arch=gfx950 -O3 tools/gap_micro.hip -o /tmp/gap_micro && /tmp/gap_micro
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }

// busy for `ticks` of the 100 MHz clock, then stamp (first, last) of the workgroup
// KA: the first stamp is taken only once the kernel arguments have arrived (as in the real
// kernels, whose first stamp follows code that reads them); otherwise s_memrealtime may issue
// before the kernel-argument loads return
#define KA_WAIT(x) do { if (KA) asm volatile("s_waitcnt lgkmcnt(0)" :: "s"(x) : "memory"); } while (0)
template <bool KA>
__global__ void __launch_bounds__(512, 1) k_scan_like(unsigned long long *st, int ticks) {
  extern __shared__ float lds[];
  KA_WAIT(ticks);
  const unsigned long long t0 = rt();
  lds[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  while ((long long)(rt() - t0) < ticks) __builtin_amdgcn_s_sleep(2);
  __syncthreads();
  if (threadIdx.x == 0) {
    st[2 * blockIdx.x] = t0;
    st[2 * blockIdx.x + 1] = rt() + (unsigned long long)lds[5] * 0;
  }
}
template <bool KA>
__global__ void __launch_bounds__(64) k_merge_like(unsigned long long *st, int ticks) {
  KA_WAIT(ticks);
  const unsigned long long t0 = rt();
  while ((long long)(rt() - t0) < ticks) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0) {
    st[2 * blockIdx.x] = t0;
    st[2 * blockIdx.x + 1] = rt();
  }
}
// the real chain's shapes: ~1.5 KiB of kernel arguments by value, and the bytes each kernel
// leaves written behind (the scan's records 1.75 MB, the merge + gather's outputs 250 KB)
struct BigArgs { unsigned long long pad[190]; int ticks; float *dirty; long long ndirty; unsigned long long *st; };
__global__ void __launch_bounds__(512, 1) k_scan_dirty(unsigned long long *st, int ticks, float *dirty, long long n) {
  extern __shared__ float lds[];
  asm volatile("s_waitcnt lgkmcnt(0)" :: "s"(ticks) : "memory");
  const unsigned long long t0 = rt();
  lds[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  while ((long long)(rt() - t0) < ticks) __builtin_amdgcn_s_sleep(2);
  for (long long i = (long long)blockIdx.x * 512 + threadIdx.x; i < n; i += (long long)gridDim.x * 512) dirty[i] = (float)i;
  __syncthreads();
  if (threadIdx.x == 0) {
    st[2 * blockIdx.x] = t0;
    st[2 * blockIdx.x + 1] = rt();
  }
}
// the scan's DB stream: every workgroup reads its 1/256 of `nbytes` (16 B per lane per load,
// 4 loads in flight), so the L2s end the launch full of clean DB lines, as the real scan leaves
// them; NT = the loads carry the non-temporal hint
typedef float f4v __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ void __launch_bounds__(512, 1) k_scan_stream(unsigned long long *st, const f4v *db, long long n4, float *sink) {
  extern __shared__ float lds[];
  asm volatile("s_waitcnt lgkmcnt(0)" :: "s"(n4) : "memory");
  const unsigned long long t0 = rt();
  lds[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  const long long per = n4 / gridDim.x, b = per * blockIdx.x;
  float acc = 0.f;
  for (long long i = threadIdx.x; i < per; i += 4 * 512) {
    f4v v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const long long j = i + u * 512;
      if (j < per) v[u] = NT ? __builtin_nontemporal_load(db + b + j) : db[b + j];
      else v[u] = f4v{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < 4; u++) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (acc == 12345.f) sink[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    st[2 * blockIdx.x] = t0;
    st[2 * blockIdx.x + 1] = rt() + (unsigned long long)lds[5] * 0;
  }
}
template <bool KA>
__global__ void __launch_bounds__(64) k_merge_big(BigArgs a) {
  KA_WAIT(a.ticks);
  const unsigned long long t0 = rt();
  while ((long long)(rt() - t0) < a.ticks) __builtin_amdgcn_s_sleep(2);
  for (long long i = (long long)blockIdx.x * 64 + threadIdx.x; i < a.ndirty; i += (long long)gridDim.x * 64) a.dirty[i] = (float)i;
  if (threadIdx.x == 0) {
    a.st[2 * blockIdx.x] = t0;
    a.st[2 * blockIdx.x + 1] = rt() + (a.pad[threadIdx.x] & 0);
  }
}

int main(int argc, char **argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 2000;
  // mode 1: the real kernels' argument size and written bytes; 2: the scan streams 120 MB
  // (L2s full of clean lines at each boundary); 6: the same with non-temporal loads; 8: mode 0
  // with the first stamps after the kernel arguments arrived (modes 1, 2, 6 always so)
  const int mode = argc > 2 ? atoi(argv[2]) : 0;
  const int nA = 256, nB = 342, ldsA = 150 * 1024;
  const int tA = 3000, tB = 1500;  // 30 / 15 us of work
  CK(hipFuncSetAttribute((const void *)k_scan_like<false>, hipFuncAttributeMaxDynamicSharedMemorySize, ldsA));
  CK(hipFuncSetAttribute((const void *)k_scan_like<true>, hipFuncAttributeMaxDynamicSharedMemorySize, ldsA));
  CK(hipFuncSetAttribute((const void *)k_scan_dirty, hipFuncAttributeMaxDynamicSharedMemorySize, ldsA));
  CK(hipFuncSetAttribute((const void *)k_scan_stream<false>, hipFuncAttributeMaxDynamicSharedMemorySize, ldsA));
  CK(hipFuncSetAttribute((const void *)k_scan_stream<true>, hipFuncAttributeMaxDynamicSharedMemorySize, ldsA));
  // mode 2: a 120 MB DB stream per scan launch (the real scan's hi bytes)
  const long long n4 = (mode & 2) ? 120000000LL / 16 : 0;
  f4v *dbs = nullptr;
  if (mode & 2) {
    CK(hipMalloc(&dbs, (size_t)n4 * 16));
    CK(hipMemset(dbs, 0, (size_t)n4 * 16));
  }
  float *dirty;
  CK(hipMalloc(&dirty, (size_t)2 << 20));
  BigArgs ba{};
  ba.ticks = 1500;
  ba.dirty = dirty;
  ba.ndirty = 250000 / 4;
  unsigned long long *st;
  const size_t per = 2 * 512;  // stamp slots per launch
  CK(hipMalloc(&st, (size_t)2 * steps * per * 8));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto enqueue = [&](int i0, int n) {
    for (int i = i0; i < i0 + n; i++) {
      if (mode & 2) {
        if (mode & 4) hipLaunchKernelGGL(k_scan_stream<true>, dim3(nA), dim3(512), ldsA, s, st + (size_t)(2 * i) * per, dbs, n4, dirty);
        else hipLaunchKernelGGL(k_scan_stream<false>, dim3(nA), dim3(512), ldsA, s, st + (size_t)(2 * i) * per, dbs, n4, dirty);
        hipLaunchKernelGGL(k_merge_like<true>, dim3(nB), dim3(64), 0, s, st + (size_t)(2 * i + 1) * per, tB);
      } else if (mode & 1) {
        hipLaunchKernelGGL(k_scan_dirty, dim3(nA), dim3(512), ldsA, s, st + (size_t)(2 * i) * per, tA, dirty, 1750000LL / 4);
        ba.st = st + (size_t)(2 * i + 1) * per;
        hipLaunchKernelGGL(k_merge_big<true>, dim3(nB), dim3(64), 0, s, ba);
      } else {
        if (mode & 8) {
          hipLaunchKernelGGL(k_scan_like<true>, dim3(nA), dim3(512), ldsA, s, st + (size_t)(2 * i) * per, tA);
          hipLaunchKernelGGL(k_merge_like<true>, dim3(nB), dim3(64), 0, s, st + (size_t)(2 * i + 1) * per, tB);
        } else {
          hipLaunchKernelGGL(k_scan_like<false>, dim3(nA), dim3(512), ldsA, s, st + (size_t)(2 * i) * per, tA);
          hipLaunchKernelGGL(k_merge_like<false>, dim3(nB), dim3(64), 0, s, st + (size_t)(2 * i + 1) * per, tB);
        }
      }
    }
  };
  auto report = [&](const char *name, double wall_ms) {
    std::vector<unsigned long long> h((size_t)2 * steps * per);
    CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
    double gAB = 0, gBA = 0, spA = 0;
    int n1 = 0, n2 = 0;
    std::vector<unsigned long long> lo(2 * steps), hi(2 * steps), smax(2 * steps);
    for (int L = 0; L < 2 * steps; L++) {
      const int n = (L & 1) ? nB : nA;
      unsigned long long a = ~0ull, b = 0, m = 0;
      for (int w = 0; w < n; w++) {
        a = std::min(a, h[(size_t)L * per + 2 * w]);
        m = std::max(m, h[(size_t)L * per + 2 * w]);
        b = std::max(b, h[(size_t)L * per + 2 * w + 1]);
      }
      lo[L] = a; hi[L] = b; smax[L] = m;
    }
    for (int L = 1; L < 2 * steps; L++) {
      const double g = (double)(lo[L] - hi[L - 1]) * 0.01;  // us
      if (L & 1) { gAB += g; n1++; } else { gBA += g; n2++; }
    }
    for (int L = 0; L < 2 * steps; L += 2) spA += (double)(smax[L] - lo[L]) * 0.01;
    printf("%-28s wall %.1f ms = %.2f us/step; gap scan->merge %.2f us, merge->scan %.2f us, scan start spread %.2f us\n",
           name, wall_ms, wall_ms * 1e3 / steps, gAB / n1, gBA / n2, spA / steps);
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms;
  // warmup
  enqueue(0, 50);
  CK(hipStreamSynchronize(s));
  // 1. eager
  CK(hipEventRecord(e0, s));
  enqueue(0, steps);
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  report("eager", ms);
  // 2. one graph of every step
  for (int chunk : {steps, 16}) {
    std::vector<hipGraphExec_t> ex;
    for (int i0 = 0; i0 < steps; i0 += chunk) {
      hipGraph_t g;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      enqueue(i0, std::min(chunk, steps - i0));
      CK(hipStreamEndCapture(s, &g));
      hipGraphExec_t x;
      CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
      CK(hipGraphDestroy(g));
      ex.push_back(x);
    }
    for (auto &x : ex) CK(hipGraphLaunch(x, s));  // warm
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (auto &x : ex) CK(hipGraphLaunch(x, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    char nm[64];
    snprintf(nm, sizeof nm, "graph (%d steps per graph)", chunk);
    report(nm, ms);
    for (auto &x : ex) CK(hipGraphExecDestroy(x));
  }
  printf("ALL-OK\n");
  return 0;
}
