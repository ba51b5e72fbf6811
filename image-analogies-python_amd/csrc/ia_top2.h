// ia_top2.h — device types shared by the MFMA distance kernels (ia_kernels.hip, ia_k3h.hip):
// MFMA operand/accumulator vectors and the per-subset top-2 record with its merge.
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>

#include "ia_internal.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));

// a K3 subset's best two (value, DB position) pairs and the threshold T: every position of
// the subset that is not listed has an MFMA value >= T
struct Top2 {
  float v1, v2, T;
  int i1, i2;
};
__device__ __forceinline__ bool lt(float va, int ia, float vb, int ib) {
  return va < vb || (va == vb && ia < ib);
}
__device__ __forceinline__ void top2_insert(Top2 &a, float v, int i, float &third) {
  if (lt(v, i, a.v1, a.i1)) {
    third = fminf(third, a.v2);
    a.v2 = a.v1; a.i2 = a.i1; a.v1 = v; a.i1 = i;
  } else if (lt(v, i, a.v2, a.i2)) {
    third = fminf(third, a.v2);
    a.v2 = v; a.i2 = i;
  } else {
    third = fminf(third, v);
  }
}
__device__ __forceinline__ Top2 top2_merge(Top2 a, const Top2 &b) {
  float third = FLT_MAX;
  top2_insert(a, b.v1, b.i1, third);
  top2_insert(a, b.v2, b.i2, third);
  a.T = fminf(fminf(a.T, b.T), third);
  return a;
}

// top2_merge without branches (selects only): the two listed pairs of a and b are each sorted, so
// the merged first is the smaller of the two heads, the second the smaller of the loser and the
// winner's second, and the third value (into T) the smaller of what remains
__device__ __forceinline__ Top2 top2_merge_sel(const Top2 &a, const Top2 &b) {
  const bool x = lt(a.v1, a.i1, b.v1, b.i1);
  const float fv = x ? a.v1 : b.v1, lv = x ? b.v1 : a.v1, nv = x ? a.v2 : b.v2, l2 = x ? b.v2 : a.v2;
  const int fi = x ? a.i1 : b.i1, li = x ? b.i1 : a.i1, ni = x ? a.i2 : b.i2;
  const bool y = lt(nv, ni, lv, li);
  Top2 r;
  r.v1 = fv;
  r.i1 = fi;
  r.v2 = y ? nv : lv;
  r.i2 = y ? ni : li;
  r.T = fminf(fminf(a.T, b.T), y ? lv : fminf(nv, l2));
  return r;
}

// v from lane (lane ^ J) for J a power of two below 64, without the LDS crossbar where the
// hardware has a register path: DPP quad_perm (J = 1, 2), ds_swizzle bit mode (4, 8),
// v_permlane16_swap (16: rows 0 <-> 1, 2 <-> 3), v_permlane32_swap (32: the two halves)
__device__ __forceinline__ unsigned xlane_xor(unsigned v, int J) {
  switch (J) {
    case 1: return (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false);
    case 2: return (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false);
    case 4: return (unsigned)__builtin_amdgcn_ds_swizzle((int)v, 0x101F);
    case 8: return (unsigned)__builtin_amdgcn_ds_swizzle((int)v, 0x201F);
    case 16: {
      const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
      return ((threadIdx.x >> 4) & 1) ? r[0] : r[1];
    }
    default: {
      const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
      return (threadIdx.x & 32) ? r[0] : r[1];
    }
  }
}
__device__ __forceinline__ float xlane_xor_f(float v, int J) { return __uint_as_float(xlane_xor(__float_as_uint(v), J)); }

// split-f16 distance kernel entry (ia_k3h.hip)
typedef void (*k3h_fn)(const h16x8 *, const h16x8 *, int, int, int, int, int, int, int, float4 *, float *);
// pruned split-f16 distance kernel entry (ia_k3h.hip, k3h_prune)
typedef void (*k3p_fn)(const h16x8 *, const h16x8 *, const float4 *, const float4 *, const int *, int, int, int, int, int,
                       float4 *, float *, unsigned long long *, unsigned long long *, int, const int *, int, int,
                       int *, const float4 *, const float *, int, int, XOScan);
