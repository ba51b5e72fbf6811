// ia_k3h.hip — K3h, the split-f16 MFMA distance scan of best_approximate_match
// (algorithms.py:73-75): |a'|^2 - 2 q'.a' for every (DB row, query) of a wavefront step on
// v_mfma_f32_32x32x16_f16 with hi/lo-split operands (ia_kernels.hip, "Split-f16 matcher"),
// fused per-query top-2 + certification threshold.
//
// Compiled once per (KS, QT) instance (-DIA_K3H_KS, -DIA_K3H_QT; see Makefile) so the
// heavily unrolled, explicitly scheduled instances build in parallel.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "ia_internal.h"
#include "ia_top2.h"

// K3h: grid = nwg workgroups of NW waves (one workgroup per CU); WG w owns DB tiles
// [w*tpw, (w+1)*tpw), wave v takes tiles w*tpw + v, +NW, ...; the step's QT query tiles sit in
// LDS (QT*KS*2 KiB); each DB tile (hi+lo, 2*KS h16x8 per lane) is loaded once into registers
// with a one-tile prefetch and contracted against every query tile: per 16 k, 3 MFMAs into one
// accumulator.  Query tiles go in pairs (two independent accumulation chains share each DB
// operand); the top-2 epilogue of pair j is issued after the MFMAs of pair j+1 (distinct
// accumulators) so it fills MFMA shadow, walking the pair's two queries in lockstep (two
// independent chains).
//
// Epilogue (per lane and query: best value b1 with its DB position, runner-up value b2):
//   PK = false: per value v (4 VALU): c = v < b1;  b2 = med3(b1, b2, v);  b1 = c ? v : b1;
//               i1 = c ? row : i1.
//   PK = true (packed index, 3 VALU per value): the value's 4 low mantissa bits are replaced
//               by its row index r within the lane's 16 rows of the tile (v_and_or_b32), so
//               min/med3 on the packed floats carry the row along:  b2 = med3(b1, b2, pv);
//               b1 = min(b1, pv); once per (query, tile): tile = (b1 changed) ? t : tile.
//               A packed value differs from the MFMA value by < 16 ulp (<= 2^-19 |v|), which
//               the certification bound includes (ia_eps_c_h(KS, true)).  f32 denormals are
//               preserved (kernel FP mode), so packed tiny values keep their index bits.
// The per-lane subsets (lane half x wave) are merged through LDS into one record per query:
// the top-2 list and the threshold T (every unlisted row of the chunk has value >= T).
template <int QT>
__device__ __forceinline__ void k3h_upd(float v, int row, int q, float (&b1)[QT], float (&b2)[QT], int (&i1)[QT]) {
  const bool c = v < b1[q];
  b2[q] = __builtin_amdgcn_fmed3f(b1[q], b2[q], v);
  b1[q] = c ? v : b1[q];
  i1[q] = c ? row : i1[q];
}
// med3 / min on packed values: single instructions (no canonicalising v_max on bit-built
// operands; the packed operands are never MFMA results, so no MFMA read hazard is hidden)
__device__ __forceinline__ float k3h_med3(float a, float b, float c) {
  float r;
  asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float k3h_min(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float k3h_pack(float v, int r) {
  return __uint_as_float((__float_as_uint(v) & ~15u) | (unsigned)r);
}

template <int QT, bool PK>
__device__ __forceinline__ void k3h_epi2(const f32x16 &e0, const f32x16 &e1, int q0, bool has1, int rb, int t,
                                         float (&b1)[QT], float (&b2)[QT], int (&i1)[QT]) {
  if constexpr (PK) {
    const float o0 = b1[q0], o1 = has1 ? b1[q0 + 1] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const float p0 = k3h_pack(e0[r], r);
      b2[q0] = k3h_med3(b1[q0], b2[q0], p0);
      b1[q0] = k3h_min(b1[q0], p0);
      if (has1) {
        const float p1 = k3h_pack(e1[r], r);
        b2[q0 + 1] = k3h_med3(b1[q0 + 1], b2[q0 + 1], p1);
        b1[q0 + 1] = k3h_min(b1[q0 + 1], p1);
      }
    }
    i1[q0] = b1[q0] != o0 ? t : i1[q0];
    if (has1) i1[q0 + 1] = b1[q0 + 1] != o1 ? t : i1[q0 + 1];
  } else {
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int row = rb + (r & 3) + 8 * (r >> 2);
      k3h_upd<QT>(e0[r], row, q0, b1, b2, i1);
      if (has1) k3h_upd<QT>(e1[r], row, q0 + 1, b1, b2, i1);
    }
  }
}

// PROBE (diagnostic builds only, never selected by the product path): 1 = epilogue reduced to
// one min per accumulator (MFMA + operand-load cost alone)
template <int KS, int QT, int NW, bool PK, int PROBE = 0>
__global__ void __launch_bounds__(NW * IA_WAVE, 1)
k3h_scan(const h16x8 *__restrict__ db, const h16x8 *__restrict__ qf, int n_tiles, int tpw, int qt0, int M, int nwg,
         int row0, int NT, float4 *__restrict__ rec, float *__restrict__ recT) {
  constexpr int NP = 2 * KS, NPAIR = (QT + 1) / 2, WGT = NW * IA_WAVE;
  extern __shared__ h16x8 ldsh[];  // QT * NP * 64 (queries), reused for the merge
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5;
  const int wg = blockIdx.x;
  const int t_begin = wg * tpw, t_end = min(n_tiles, t_begin + tpw);
  int t = t_begin + wave;

  h16x8 a[NP], an[NP];
  {  // first DB tile: requested before the query fill so both latencies overlap
    const h16x8 *src = db + (int64_t)min(t, n_tiles - 1) * NP * IA_WAVE + lane;
#pragma unroll
    for (int p = 0; p < NP; p++) a[p] = src[p * IA_WAVE];
  }
  const h16x8 *qsrc = qf + (int64_t)qt0 * NP * IA_WAVE;
  for (int i = threadIdx.x; i < QT * NP * IA_WAVE; i += WGT) ldsh[i] = qsrc[i];
  __syncthreads();

  float b1[QT], b2[QT];
  int i1[QT];  // PK = false: DB position of b1;  PK = true: tile of b1
#pragma unroll
  for (int q = 0; q < QT; q++) {
    b1[q] = FLT_MAX;
    b2[q] = FLT_MAX;
    i1[q] = 0x7fffffff;
  }
  for (; t < t_end; t += NW) {
    {  // prefetch the next tile of this wave (clamped: always issue, never branch per load)
      const h16x8 *src = db + (int64_t)min(t + NW, n_tiles - 1) * NP * IA_WAVE + lane;
#pragma unroll
      for (int p = 0; p < NP; p++) an[p] = src[p * IA_WAVE];
    }
    const int rbase = row0 + t * IA_TILE + 4 * half;
    asm volatile("" ::: "memory");  // LDS query fragments are re-read per tile, not hoisted
    f32x16 e0, e1;
#pragma unroll
    for (int qp = 0; qp < NPAIR; qp++) {
      constexpr f32x16 zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const bool two = 2 * qp + 1 < QT;
      f32x16 c0 = zero, c1 = zero;
      const h16x8 *qb0 = ldsh + (2 * qp) * NP * IA_WAVE + lane;
      const h16x8 *qb1 = qb0 + NP * IA_WAVE;
#pragma unroll
      for (int s = 0; s < KS; s++) {
        const h16x8 x0h = qb0[(2 * s) * IA_WAVE], x0l = qb0[(2 * s + 1) * IA_WAVE];
        const h16x8 x1h = two ? qb1[(2 * s) * IA_WAVE] : x0h, x1l = two ? qb1[(2 * s + 1) * IA_WAVE] : x0l;
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s + 1], x0h, c0, 0, 0, 0);
        if (two) c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s + 1], x1h, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], x0l, c0, 0, 0, 0);
        if (two) c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], x1l, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], x0h, c0, 0, 0, 0);
        if (two) c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], x1h, c1, 0, 0, 0);
      }
      if constexpr (PROBE == 1) {
        b1[2 * qp] = fminf(b1[2 * qp], c0[qp & 15]);
        if (two) b1[2 * qp + 1] = fminf(b1[2 * qp + 1], c1[qp & 15]);
      } else {
        if (qp >= 1) k3h_epi2<QT, PK>(e0, e1, 2 * qp - 2, true, rbase, t, b1, b2, i1);
        e0 = c0;
        e1 = c1;
      }
    }
    if constexpr (PROBE == 0) k3h_epi2<QT, PK>(e0, e1, 2 * (NPAIR - 1), 2 * NPAIR - 1 < QT, rbase, t, b1, b2, i1);
#pragma unroll
    for (int p = 0; p < NP; p++) a[p] = an[p];
  }
  if constexpr (PK) {  // tile + packed in-tile index -> DB position
#pragma unroll
    for (int q = 0; q < QT; q++) {
      const int r = (int)(__float_as_uint(b1[q]) & 15u);
      i1[q] = b1[q] == FLT_MAX ? 0x7fffffff : row0 + i1[q] * IA_TILE + 4 * half + (r & 3) + 8 * (r >> 2);
    }
  }

  // ---- merge the 2*NW subsets of each query: lane halves by shuffle, waves through LDS
  __syncthreads();
  Top2 *red = reinterpret_cast<Top2 *>(ldsh);  // [NW][QT][32]
#pragma unroll
  for (int q = 0; q < QT; q++) {
    Top2 mine = {b1[q], FLT_MAX, b2[q], i1[q], 0x7fffffff};
    Top2 other;
    other.v1 = __shfl_xor(b1[q], 32, 64);
    other.i1 = __shfl_xor(i1[q], 32, 64);
    other.T = __shfl_xor(b2[q], 32, 64);
    other.v2 = FLT_MAX;
    other.i2 = 0x7fffffff;
    Top2 mrg = half == 0 ? top2_merge(mine, other) : top2_merge(other, mine);
    if (half == 0) red[(wave * QT + q) * IA_TILE + lane] = mrg;
  }
  __syncthreads();
  for (int x = threadIdx.x; x < QT * IA_TILE; x += WGT) {
    Top2 m = red[x];
#pragma unroll
    for (int w = 1; w < NW; w++) m = top2_merge(m, red[(w * QT) * IA_TILE + x]);
    const int qg = qt0 * IA_TILE + x;
    if (qg < M) {  // positions -> DB rows (ia_pos_row); never-set entries stay out of range
      const int r1 = m.i1 == 0x7fffffff ? m.i1 : (int)ia_pos_row(m.i1, NT);
      const int r2 = m.i2 == 0x7fffffff ? m.i2 : (int)ia_pos_row(m.i2, NT);
      rec[(int64_t)qg * nwg + wg] = make_float4(m.v1, __int_as_float(r1), m.v2, __int_as_float(r2));
      recT[(int64_t)qg * nwg + wg] = m.T;
    }
  }
}

#if defined(IA_K3H_KS) && defined(IA_K3H_QT)
#define IA_K3H_CAT2(a, b, c) a##b##_##c
#define IA_K3H_CAT(a, b, c) IA_K3H_CAT2(a, b, c)
// variant (option "k3_variant"): 0 = compare/select epilogue, 1 = packed-index epilogue
k3h_fn IA_K3H_CAT(ia_k3h_get_, IA_K3H_KS, IA_K3H_QT)(int variant) {
  if (variant == 1) return k3h_scan<IA_K3H_KS, IA_K3H_QT, IA_WGH / IA_WAVE, true>;
#ifdef IA_K3H_DIAG  // diagnostic variants (plateau instance only)
  if constexpr (IA_K3H_KS == 4 && IA_K3H_QT == 11) {
    if (variant == 2) return k3h_scan<IA_K3H_KS, IA_K3H_QT, 4, true>;
    if (variant == 3) return k3h_scan<IA_K3H_KS, IA_K3H_QT, IA_WGH / IA_WAVE, true, 1>;
  }
#endif
  return k3h_scan<IA_K3H_KS, IA_K3H_QT, IA_WGH / IA_WAVE, false>;
}
#endif
