// ia_prune.hip — per-level setup of the certified pruned distance scan.
//
// The exact NN of a query q can only be a DB row a with |a - q|^2 <= U, U = the exact fp64
// distance of q's best coherence candidate (itself a DB row).  For an orthonormal basis u_1..u_k
// of R^D, sum_i (u_i . (a - q))^2 <= |a - q|^2, so a row whose projection box lies further than
// sqrt(U) from q's projection can be skipped without changing the result.  Per level:
//   K5a/K5b  covariance of the centred fp64 DB rows (sampled, deterministic two-pass reduction);
//            the host takes its top IA_NPC eigenvectors (Jacobi, ia_capi.cpp) as the basis
//   K5c      projections of every row onto the basis + a Morton key of the quantised
//            projections; hipCUB radix sort of (key, row) orders the DB so that 32-row tiles
//            are compact in projection space
//   K5d      position -> row table (sort neighbours alternate between the two lane halves of
//            a tile, i.e. between K3 subsets) and per-tile projection boxes (fp32, rounded
//            outward)
// Only the 1-channel split-f16 path prunes (the bench configuration); everything else scans.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <float.h>
#include <math.h>
#include <stdint.h>

#include "ia_internal.h"
#include "ia_launch.h"
#include "ia_prune.h"
#include "ia_top2.h"

#define PR_WG 256
#define PR_COV_ROWS 16  // rows staged in LDS per covariance pass

__device__ __forceinline__ int prune_part1(int f) { return f < 9 ? 0 : f < 34 ? 1 : f < 43 ? 2 : 3; }

// K5a: partial sums of x'_f x'_g (f <= g) over the sampled rows r = (wg + nwg*k) * stride
__global__ void __launch_bounds__(PR_WG) k_cov_partial(const double *__restrict__ db64, int64_t NA, int64_t stride,
                                                       const double *__restrict__ mu_part, double *__restrict__ part) {
  constexpr int D = 55, DS = 56, NPAIR = D * (D + 1) / 2, PPT = (NPAIR + PR_WG - 1) / PR_WG;
  __shared__ double xs[PR_COV_ROWS][DS];
  int pf[PPT], pg[PPT];
  double acc[PPT];
#pragma unroll
  for (int k = 0; k < PPT; k++) {
    int p = threadIdx.x + PR_WG * k, f = 0;
    if (p >= NPAIR) p = NPAIR - 1;
    while (p >= D - f) {  // pair p -> (f, g), f <= g, row-major upper triangle
      p -= D - f;
      f++;
    }
    pf[k] = f;
    pg[k] = f + p;
    acc[k] = 0.;
  }
  const int64_t nsamp = (NA + stride - 1) / stride;
  for (int64_t base = (int64_t)blockIdx.x * PR_COV_ROWS; base < nsamp; base += (int64_t)gridDim.x * PR_COV_ROWS) {
    for (int i = threadIdx.x; i < PR_COV_ROWS * DS; i += PR_WG) {
      const int rr = i / DS, f = i % DS;
      const int64_t s = base + rr;
      double v = 0.;
      if (s < nsamp && f < D) v = db64[s * stride * DS + f] - mu_part[prune_part1(f)];
      xs[rr][f] = v;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PPT; k++) {
#pragma unroll 4
      for (int rr = 0; rr < PR_COV_ROWS; rr++) acc[k] += xs[rr][pf[k]] * xs[rr][pg[k]];
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < PPT; k++) {
    const int p = threadIdx.x + PR_WG * k;
    if (p < NPAIR) part[(int64_t)blockIdx.x * NPAIR + p] = acc[k];
  }
}

// K5b: fixed-order sum of the partials, one thread per pair (25 one-wave workgroups: the
// partials of adjacent pairs are adjacent, so every load of a wave is one coalesced row)
__global__ void __launch_bounds__(64) k_cov_reduce(const double *__restrict__ part, int nwg, double *__restrict__ cov) {
  constexpr int NPAIR = 55 * 56 / 2;
  const int p = blockIdx.x * 64 + threadIdx.x;
  if (p >= NPAIR) return;
  double s = 0.;
#pragma unroll 8
  for (int w = 0; w < nwg; w++) s += part[(int64_t)w * NPAIR + p];
  cov[p] = s;
}

// K5c: projections, keys and the identity row list of every DB row
__global__ void __launch_bounds__(PR_WG) k_proj_keys(const double *__restrict__ db64, int64_t NA,
                                                     const double *__restrict__ mu_part, const double *__restrict__ basis,
                                                     double *__restrict__ proj, unsigned *__restrict__ keys,
                                                     int *__restrict__ rows, float *__restrict__ rnorm) {
  constexpr int D = 55, DS = 56;
  __shared__ double ub[IA_NPC * D + IA_NPC];
  for (int i = threadIdx.x; i < IA_NPC * D + IA_NPC; i += PR_WG) ub[i] = basis[i];
  __syncthreads();
  const int64_t row = (int64_t)blockIdx.x * PR_WG + threadIdx.x;
  if (row >= NA) return;
  const double2 *a2 = reinterpret_cast<const double2 *>(db64 + row * DS);
  double p[IA_NPC], n2 = 0.;
#pragma unroll
  for (int i = 0; i < IA_NPC; i++) p[i] = 0.;
#pragma unroll
  for (int k = 0; k < DS / 2; k++) {
    const double2 v = a2[k];
    const int f0 = 2 * k, f1 = 2 * k + 1;
    const double x0 = v.x - mu_part[prune_part1(f0)];
    n2 += x0 * x0;
#pragma unroll
    for (int i = 0; i < IA_NPC; i++) p[i] += ub[i * D + f0] * x0;
    if (f1 < D) {
      const double x1 = v.y - mu_part[prune_part1(f1)];
      n2 += x1 * x1;
#pragma unroll
      for (int i = 0; i < IA_NPC; i++) p[i] += ub[i * D + f1] * x1;
    }
  }
  // |a'| (the centred row of the split-f16 DB, k_db_build_h), rounded up: fp64 sum and sqrt
  // err by < 2^-46 relative, covered by the (1 + 2^-40) factor
  rnorm[row] = round_up_f(sqrt(n2) * (1.0 + 0x1p-40));
#pragma unroll
  for (int i = 0; i < IA_NPC; i++) proj[row * IA_NPC + i] = p[i];
  keys[row] = prune_key(p, ub + IA_NPC * D);
  rows[row] = (int)row;
}

// K5d: position -> row table.  Sorted index k of tile t sits in slot ((k >> 1) & 3) +
// 8 * (k >> 3) + 4 * (k & 1): consecutive sorted rows alternate between the lane halves of the
// MFMA output (half = (slot >> 2) & 1), i.e. between K3 subsets.  Positions past NA map to
// rows >= NA (padding: never a candidate).
// G > 1 (option "prune_group"): the Morton tiles of each full group of G hold the group's G x 32
// sorted rows interleaved (tile r of the group: sorted rows r, r + G, r + 2G, ...), so sort
// neighbours - near-duplicate rows - land in different tiles and hence in different K3p
// workgroup chunks (tiles r, r + 1 of a group belong to chunks w, w + 1), where their near-tied
// distances cannot leave a chunk's threshold within epsilon of its winner; a trailing partial
// group keeps G = 1.  (The boxes follow the rows, so they grow with G.)
// Shards (W > 1, DB sharded over W ranks): Morton tile m belongs to shard m mod W, and the
// storage order groups each shard's tiles contiguously (shard r: storage tiles [off_r, off_r +
// NT_r), NT_r = ceil((NT - r) / W), local tile k = Morton tile r + W k).  Every shard thus
// covers the whole feature space evenly (balanced pruned work) and is a contiguous range of
// the DB, the table and the boxes.
__global__ void __launch_bounds__(PR_WG) k_make_table(const int *__restrict__ sorted_rows, int64_t NA, int n_tiles, int W,
                                                      int G, int *__restrict__ pos2row) {
  const int64_t p = (int64_t)blockIdx.x * PR_WG + threadIdx.x;
  if (p >= (int64_t)n_tiles * IA_TILE) return;
  const int j = (int)(p & 31);
  const int k = (((j & 3) << 1) | ((j >> 2) & 1) | ((j >> 3) << 3));
  const int64_t tm = W > 1 ? ia_shard_morton_tile_(p >> 5, n_tiles, W) : (p >> 5);
  const int64_t grp = tm / G;
  const int64_t s = (grp + 1) * G <= n_tiles ? grp * G * IA_TILE + (int64_t)k * G + (tm - grp * G) : tm * IA_TILE + k;
  pos2row[p] = s < NA ? sorted_rows[s] : (int)s;
}

// K5d': per-tile boxes of the projections (lo[IA_NPC], hi[IA_NPC]) over the tile's real rows
__global__ void __launch_bounds__(PR_WG) k_tile_boxes(const int *__restrict__ pos2row, const double *__restrict__ proj,
                                                      int64_t NA, int n_tiles, float *__restrict__ boxes,
                                                      const float *__restrict__ rnorm, float *__restrict__ tnorm) {
  const int t = blockIdx.x * PR_WG + threadIdx.x;
  if (t >= n_tiles) return;
  double lo[IA_NPC], hi[IA_NPC];
#pragma unroll
  for (int i = 0; i < IA_NPC; i++) {
    lo[i] = DBL_MAX;
    hi[i] = -DBL_MAX;
  }
  float rt = 0.f;  // R_t = max |a'| over the tile's real rows (K3p's hi x hi filter, k3p_variant 14/15)
  for (int j = 0; j < IA_TILE; j++) {
    const int row = pos2row[(int64_t)t * IA_TILE + j];
    if (row >= NA) continue;
    rt = fmaxf(rt, rnorm[row]);
#pragma unroll
    for (int i = 0; i < IA_NPC; i++) {
      const double v = proj[(int64_t)row * IA_NPC + i];
      lo[i] = fmin(lo[i], v);
      hi[i] = fmax(hi[i], v);
    }
  }
#pragma unroll
  for (int i = 0; i < IA_NPC; i++) {
    const bool empty = lo[i] > hi[i];
    boxes[(int64_t)t * 2 * IA_NPC + i] = empty ? INFINITY : round_down_f(lo[i]);
    boxes[(int64_t)t * 2 * IA_NPC + IA_NPC + i] = empty ? -INFINITY : round_up_f(hi[i]);
  }
  tnorm[t] = rt;
}

// K2s: one sort of a wavefront step's queries for the pruned scan (k3p_variant 11).  One
// workgroup per sorted query tile: each sorts the step's unique keys (the Morton key's top 20
// bits above the 12-bit query index; padding slots and unused sort slots last) by a bitonic
// network in LDS - the same order in every workgroup - and writes its tile's pruning records,
// split-f16 fragments and box (min lo, max hi, max U' over its real queries) in sorted order,
// so every K3p launch loads just its slice.  Any Mpad <= 4096 (the in-kernel sort of K3p v6/v7
// is limited to 512).  (One workgroup for the whole step spent 20.7 us per cfg4 step, mostly
// in the copies.)
#define QS_WG 1024
// XO (owner-computes sharded step, option "exchange" = 2, ia_internal.h XOSort): the owner's Mj
// queries [q0, q0 + Mj) of the local K2p output are sorted alone (local index in the key's low
// 12 bits), its QTs tiles go to tiles [tile0, tile0 + QTs) of every rank's exchange area (slots
// past Mj: padding, U' = -inf, never contracted, no record), each followed by its flag = seq.
template <bool XO>
__global__ void __launch_bounds__(QS_WG) k_query_sort(const float4 *__restrict__ qinfo, const h16x8 *__restrict__ qf,
                                                      int Mpad, int NS, int NP, int *__restrict__ order,
                                                      float4 *__restrict__ sq, h16x8 *__restrict__ qfs,
                                                      float4 *__restrict__ tbox, XOSort xs) {
  __shared__ unsigned key[4096];
  const int tid = threadIdx.x;
  // sort key of sort slot i: unique (query index in the low 12 bits); padding last
  auto key_of = [&](int i) -> unsigned {
    if constexpr (XO) return i < xs.Mj ? ((__float_as_uint(qinfo[3 * (xs.q0 + i) + 2].y) & 0xFFFFF000u) | (unsigned)i) : 0xFFFFFFFFu;
    else return i < Mpad ? ((__float_as_uint(qinfo[3 * i + 2].y) & 0xFFFFF000u) | (unsigned)i) : 0xFFFFFFFFu;
  };
  if (NS <= QS_WG) {
    // one key per thread: exchanges below distance 64 are lane shuffles (no barrier), the wider
    // ones go through LDS
    unsigned v = key_of(tid);
    for (int k = 2; k <= NS; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        unsigned o;
        if (j >= 64) {
          key[tid] = v;
          __syncthreads();
          o = key[tid ^ j];
          __syncthreads();
        } else {
          o = (unsigned)__shfl_xor((int)v, j, 64);
        }
        const bool keep_min = ((tid & k) == 0) == ((tid & j) == 0);
        v = keep_min ? min(v, o) : max(v, o);
      }
    }
    key[tid] = v;
    __syncthreads();
  } else {
    for (int i = tid; i < NS; i += QS_WG) key[i] = key_of(i);
    __syncthreads();
    for (int k = 2; k <= NS; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < NS / 2; i += QS_WG) {
          const int lo = 2 * i - (i & (j - 1)), hi = lo + j;
          const unsigned a = key[lo], b = key[hi];
          const bool up = (lo & k) == 0;
          if ((a > b) == up) {
            key[lo] = b;
            key[hi] = a;
          }
        }
        __syncthreads();
      }
    }
  }
  const int xt0 = blockIdx.x;  // this workgroup's sorted query tile
  const int nout = XO ? xs.W : 1;
  // query (in qinfo / qf) of sorted slot x, -1 for XO padding
  auto q_of = [&](int x) -> int {
    const unsigned k = key[x];
    if constexpr (XO) return k == 0xFFFFFFFFu ? -1 : xs.q0 + (int)(k & 0xFFFu);
    else return (int)(k & 0xFFFu);
  };
  const int dt = XO ? xs.tile0 : 0;  // output tile offset
  for (int x = xt0 * IA_TILE + tid; x < (xt0 + 1) * IA_TILE && tid < IA_TILE; x += QS_WG) {
    const int q = q_of(x);
    const float4 i0 = q >= 0 ? qinfo[3 * q] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 i1 = q >= 0 ? qinfo[3 * q + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 i2 = q >= 0 ? qinfo[3 * q + 2] : make_float4(-INFINITY, 0.f, -INFINITY, 0.f);
    const int ov = XO ? (q >= 0 ? q - xs.q0 : 0x7fffffff) : q;
    if (XO && q >= 0) xs.inv[dt * IA_TILE + (q - xs.q0)] = dt * IA_TILE + x;  // the owner's query -> slot
    for (int o = 0; o < nout; o++) {
      const int xo = dt * IA_TILE + x;
      int *ord = XO ? reinterpret_cast<int *>(xs.area[o] + XOLayout::ORD) : order;
      float4 *si = XO ? reinterpret_cast<float4 *>(xs.area[o] + XOLayout::INFO) : sq;
      ord[xo] = ov;
      si[3 * xo] = i0;
      si[3 * xo + 1] = i1;
      si[3 * xo + 2] = i2;
    }
  }
  // fragments of the tile: sorted slot x of tile xt, piece p, lane L (k-half L >> 5, row L & 31)
  for (int e = xt0 * NP * IA_WAVE + tid; e < (xt0 + 1) * NP * IA_WAVE; e += QS_WG) {
    const int L = e & 63, pq = e >> 6, xt = pq / NP, p = pq - xt * NP;
    const int q = q_of(xt * IA_TILE + (L & 31));
    const h16x8 v = q >= 0 ? qf[((q >> 5) * NP + p) * IA_WAVE + (L & 32) + (q & 31)] : h16x8{};
    for (int o = 0; o < nout; o++) {
      h16x8 *dst = XO ? reinterpret_cast<h16x8 *>(xs.area[o] + XOLayout::FRAG) : qfs;
      dst[(int64_t)dt * NP * IA_WAVE + e] = v;
    }
  }
  // the tile's box: one 32-lane half-wave
  const int lane = tid & 63;
  for (int t = xt0 + (tid >> 5); t < xt0 + 1; t += QS_WG / 32) {
    const int q = q_of(t * IA_TILE + (lane & 31));
    const float4 u = q >= 0 ? qinfo[3 * q + 2] : make_float4(-INFINITY, 0.f, 0.f, 0.f);
    float4 lo = make_float4(INFINITY, INFINITY, INFINITY, INFINITY), hi = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    float um = -INFINITY;
    if (u.x != -INFINITY) {  // padding slots (U' = -inf) never widen a box
      lo = qinfo[3 * q];
      hi = qinfo[3 * q + 1];
      um = u.x;
    }
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      lo.x = fminf(lo.x, __shfl_xor(lo.x, o, 64));
      lo.y = fminf(lo.y, __shfl_xor(lo.y, o, 64));
      lo.z = fminf(lo.z, __shfl_xor(lo.z, o, 64));
      lo.w = fminf(lo.w, __shfl_xor(lo.w, o, 64));
      hi.x = fmaxf(hi.x, __shfl_xor(hi.x, o, 64));
      hi.y = fmaxf(hi.y, __shfl_xor(hi.y, o, 64));
      hi.z = fmaxf(hi.z, __shfl_xor(hi.z, o, 64));
      hi.w = fmaxf(hi.w, __shfl_xor(hi.w, o, 64));
      um = fmaxf(um, __shfl_xor(um, o, 64));
    }
    if ((lane & 31) == 0) {
      for (int o = 0; o < nout; o++) {
        float4 *tb = XO ? reinterpret_cast<float4 *>(xs.area[o] + XOLayout::TBOX) : tbox;
        tb[3 * (dt + t)] = lo;
        tb[3 * (dt + t) + 1] = hi;
        tb[3 * (dt + t) + 2] = make_float4(um, 0.f, 0.f, 0.f);
      }
    }
  }
  if constexpr (XO) {
    // every store of this workgroup reaches every rank before the tile's flag: each wave waits
    // for its own (uncached) stores to complete, the barrier orders them before the flag stores
    ia_stores_done();
    __syncthreads();
    if (tid < nout) {
      unsigned *fl = reinterpret_cast<unsigned *>(xs.area[tid] + XOLayout::FLAG);
      __hip_atomic_store(fl + dt + xt0, xs.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}


// ---- host launchers ---------------------------------------------------------------------------
void ia_launch_query_sort(const float4 *qinfo, const void *qf, int Mpad, int KS, int *order, float4 *sq, void *qfs,
                          float4 *tbox, hipStream_t st) {
  int NS = 32;
  while (NS < Mpad) NS <<= 1;
  hipLaunchKernelGGL(k_query_sort<false>, dim3(Mpad / IA_TILE), dim3(QS_WG), 0, st, qinfo, (const h16x8 *)qf, Mpad, NS,
                     2 * KS, order, sq, (h16x8 *)qfs, tbox, XOSort{});
}
void ia_launch_query_sort_xo(const float4 *qinfo, const void *qf, const XOSort &xs, hipStream_t st) {
  int NS = 32;
  while (NS < xs.QTs * IA_TILE) NS <<= 1;
  hipLaunchKernelGGL(k_query_sort<true>, dim3(xs.QTs), dim3(QS_WG), 0, st, qinfo, (const h16x8 *)qf, xs.QTs * IA_TILE, NS, 8,
                     nullptr, nullptr, nullptr, nullptr, xs);
}
static inline unsigned pr_cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

void ia_launch_cov(const double *db64, int64_t NA, int64_t stride, int nwg, const double *mu_part, double *part,
                   double *cov, hipStream_t st) {
  hipLaunchKernelGGL(k_cov_partial, dim3(nwg), dim3(PR_WG), 0, st, db64, NA, stride, mu_part, part);
  hipLaunchKernelGGL(k_cov_reduce, dim3(pr_cdiv(55 * 56 / 2, 64)), dim3(64), 0, st, part, nwg, cov);
}

void ia_launch_proj_keys(const double *db64, int64_t NA, const double *mu_part, const double *basis, double *proj,
                         unsigned *keys, int *rows, float *rnorm, hipStream_t st) {
  hipLaunchKernelGGL(k_proj_keys, dim3(pr_cdiv(NA, PR_WG)), dim3(PR_WG), 0, st, db64, NA, mu_part, basis, proj, keys, rows,
                     rnorm);
}

size_t ia_sort_temp_bytes(int64_t n) {
  size_t bytes = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const unsigned *)nullptr, (unsigned *)nullptr, (const int *)nullptr,
                                     (int *)nullptr, (int)n, 0, 32, (hipStream_t)0);
  return bytes;
}

int ia_sort_pairs(void *temp, size_t temp_bytes, const unsigned *keys_in, unsigned *keys_out, const int *vals_in,
                  int *vals_out, int64_t n, hipStream_t st) {
  return (int)hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, vals_in, vals_out, (int)n, 0, 32, st);
}

void ia_launch_table_boxes(const int *sorted_rows, const double *proj, int64_t NA, int n_tiles, int W, int G, int *pos2row,
                           float *boxes, const float *rnorm, float *tnorm, hipStream_t st) {
  hipLaunchKernelGGL(k_make_table, dim3(pr_cdiv((int64_t)n_tiles * IA_TILE, PR_WG)), dim3(PR_WG), 0, st, sorted_rows, NA,
                     n_tiles, W, G, pos2row);
  hipLaunchKernelGGL(k_tile_boxes, dim3(pr_cdiv(n_tiles, PR_WG)), dim3(PR_WG), 0, st, pos2row, proj, NA, n_tiles, boxes,
                     rnorm, tnorm);
}

