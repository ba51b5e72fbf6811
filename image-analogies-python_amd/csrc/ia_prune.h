// ia_prune.h — device helpers of the certified pruned distance scan, shared by
// the per-level setup (ia_prune.hip), the query gather K2p (ia_kernels.hip) and the pruned
// MFMA scan K3p (ia_k3h.hip).
//
// Bound: for orthonormal u_1..u_k and a DB row a, sum_i (u_i . (a - q))^2 <= |a - q|^2, and
// u_i . a lies in the [lo_i, hi_i] box of a's tile, so
//     LB(q, tile) = sum_i max(lo_i - qhi_i, qlo_i - hi_i, 0)^2 <= |a - q|^2  for every row a,
// with [qlo_i, qhi_i] an f32 interval around q's projection.  A (DB tile, query) pair whose LB
// exceeds U' (an f32 upper bound of the distance of the query's best coherence candidate, a DB
// row, plus a relative separation margin) cannot hold the exact NN nor tie it.
//   * projections are fp64 (error <= 55 * 2^-53 * |x| < 6e-12 for |x| <= 128 sqrt(55), the
//     f16 gate IA_F16_MAXABS); the query interval is widened by IA_PRUNE_MABS = 2^-30 on both
//     sides and rounded outward, tile boxes are rounded outward
//   * the f32 LB evaluation errs by < 2^-21 relative; the basis' deviation from orthonormality
//     delta (host, Gershgorin on U^T U) and a 2^-19 separation margin enter U':
//         U' = round_up_f32(U * (1 + delta) * (1 + 2^-17) * (1 + 2^-19))
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include "ia_internal.h"

static_assert(IA_NPC == 4, "pruning records hold 4 projections (float4)");

#define IA_PRUNE_MABS 9.313225746154785e-10  // 2^-30
#define IA_PRUNE_KEY_MAX 0xFFFFFFFDu         // real queries / DB rows with a finite bound
#define IA_PRUNE_KEY_INF 0xFFFFFFFEu         // queries without a coherence candidate (U' = inf)
#define IA_PRUNE_KEY_PAD 0xFFFFFFFFu         // padding query slots (U' = -inf: never need a tile)

__device__ __forceinline__ float round_down_f(double x) {
  float f = (float)x;
  if ((double)f > x) f = nextafterf(f, -INFINITY);
  return f;
}
__device__ __forceinline__ float round_up_f(double x) {
  float f = (float)x;
  if ((double)f < x) f = nextafterf(f, INFINITY);
  return f;
}

// Morton key of the projections quantised to 8 bits each over [-4 sigma_i, 4 sigma_i]
// (scale_i = 1 / (4 sigma_i)); DB rows and queries use the same key
__device__ __forceinline__ unsigned prune_key(const double (&p)[IA_NPC], const double *__restrict__ scale) {
  unsigned qv[IA_NPC];
#pragma unroll
  for (int i = 0; i < IA_NPC; i++) {
    const double t = (p[i] * scale[i] + 1.0) * 128.0;
    qv[i] = t <= 0. ? 0u : t >= 255. ? 255u : (unsigned)t;
  }
  // bit b of qv[i] goes to bit 4 b + 3 - i (Morton order, axis 0 most significant): each 8-bit
  // coordinate spread to every fourth bit by three shift-and-mask steps
  auto spread = [](unsigned x) {
    x = (x | (x << 12)) & 0x000F000Fu;
    x = (x | (x << 6)) & 0x03030303u;
    return (x | (x << 3)) & 0x11111111u;
  };
  const unsigned key = (spread(qv[0]) << 3) | (spread(qv[1]) << 2) | (spread(qv[2]) << 1) | spread(qv[3]);
  return key < IA_PRUNE_KEY_MAX ? key : IA_PRUNE_KEY_MAX;
}

// f32 lower bound of |a - q|^2 over the rows of a box (lo, hi) for the query interval (ql, qh)
__device__ __forceinline__ float prune_lb(const float4 &lo, const float4 &hi, const float4 &ql, const float4 &qh) {
  const float g0 = fmaxf(fmaxf(lo.x - qh.x, ql.x - hi.x), 0.f);
  const float g1 = fmaxf(fmaxf(lo.y - qh.y, ql.y - hi.y), 0.f);
  const float g2 = fmaxf(fmaxf(lo.z - qh.z, ql.z - hi.z), 0.f);
  const float g3 = fmaxf(fmaxf(lo.w - qh.w, ql.w - hi.w), 0.f);
  return fmaf(g3, g3, fmaf(g2, g2, fmaf(g1, g1, g0 * g0)));
}
