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
#include <stdio.h>

#include "ia_internal.h"
#include "ia_top2.h"
#include "ia_prune.h"

template <int KS>
__device__ __forceinline__ void ld_tile(h16x8 (&a)[2 * KS], const h16x8 *__restrict__ db, int64_t tile, int lane) {
  const h16x8 *src = db + tile * TileFmt<KS>::STRIDE;
#pragma unroll
  for (int p = 0; p < 2 * KS; p++) a[p] = src[TileFmt<KS>::off(p, lane)];
}
// the hi pieces (2s) of a tile only: half its bytes (k3p_variant 22 / 23)
template <int KS>
__device__ __forceinline__ void ld_hi(h16x8 (&h)[KS], const h16x8 *__restrict__ db, int64_t tile, int lane) {
  const h16x8 *src = db + tile * TileFmt<KS>::STRIDE;
#pragma unroll
  for (int s = 0; s < KS; s++) h[s] = src[TileFmt<KS>::off(2 * s, lane)];
}

// k3p_variant 24 / 25: the hi pieces of a tile by LDS-DMA (global_load_lds_dwordx4) into a
// 3.5 KiB slot of the wave's ring in LDS: pieces 0, 2, 4 (1 KiB, every lane) at slot + 0, 1, 2
// KiB, the compact piece 6 (512 B, lanes 0-31) at slot + 3 KiB.  Four vector-memory operations
// per tile, issued by inline asm: the compiler then neither knows of the pending LDS writes nor
// inserts its own (vmcnt(0)) waits before LDS accesses it cannot prove disjoint from them; the
// consumer waits with an explicit s_waitcnt vmcnt before it reads a slot (ring_wait, which
// clobbers "memory", so no LDS read is scheduled above it).  The DMAs write LDS only, never a
// register, so nothing the register allocator does can observe them early.
//
// Two rules this asm must keep (both broke once in round 5):
//  * M0-offset rule: an LDS-DMA's immediate offset is added to the LDS destination (M0) as well
//    as to the global address.  dma16 therefore takes no offset at all: the piece steps are in
//    the per-lane global pointer and in lds_addr, and the instruction's offset field is 0 ("off",
//    no offset:) - a saddr form with the piece steps in the immediate made the slots overlap and
//    run past the ring (a memory-aperture fault, profiles/r05/saddr/pytest_first_form_fault.log).
//  * MFMA -> VALU hazard rule: hipcc pads no wait states inside an asm statement, so no asm in this
//    file reads an MFMA result (a v_min3_f32 in asm on the filter's accumulators read stale values;
//    the filter's minimum is compiler code, k3p_min16).  The asm v_min / v_med3 of the epilogue
//    read only packed values built by VALU code from the accumulators (k3h_pack), whose MFMA hazard
//    the compiler already padded.
typedef unsigned v4u32 __attribute__((ext_vector_type(4)));  // 16-B buffer store payload
#define IA_HSLOT 224  // h16x8 per ring slot (3.5 KiB)
static_assert(3 * 1024 + 512 == IA_HSLOT * 16, "a slot holds pieces 0, 2, 4 (1 KiB each) and the compact piece 6");
__device__ __forceinline__ void dma16(const void *g, unsigned lds_addr) {
#ifdef IA_EXP_DMA_NT  // experiment: the hi stream's DMAs with the non-temporal policy
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt" ::"s"(lds_addr), "v"(g) : "memory", "m0");
#else
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds_addr), "v"(g) : "memory", "m0");
#endif
}
template <int KS>
__device__ __forceinline__ void dma_hi(const h16x8 *__restrict__ db, int64_t tile, h16x8 *slot, int lane) {
  static_assert(KS == 4, "ring slots hold compact 1-channel tiles");
  const h16x8 *src = db + tile * TileFmt<KS>::STRIDE;
  const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) h16x8 *)slot;
#pragma unroll
  for (int s = 0; s < 3; s++) dma16(src + TileFmt<KS>::off(2 * s, lane), base + s * 1024u);
  if (lane < 32) dma16(src + TileFmt<KS>::off(6, lane), base + 3072u);
}
template <int N>
__device__ __forceinline__ void ring_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// the MFMA A operand (hi pieces) of a ring slot: piece 6's upper-half lanes repeat the lower half
__device__ __forceinline__ void slot_hi(h16x8 (&h)[4], const h16x8 *slot, int lane) {
  h[0] = slot[lane];
  h[1] = slot[IA_WAVE + lane];
  h[2] = slot[2 * IA_WAVE + lane];
  h[3] = slot[3 * IA_WAVE + (lane & 31)];
}

#ifndef IA_PROBE
#define IA_PROBE 0
#endif
#if IA_PROBE & 16  // diagnostic build only: per-wave phase cycle sums of the pruned scan (K3p, V >= 1)
__device__ unsigned long long k3p_prof[24];
#define K3P_T(x) do { __builtin_amdgcn_sched_barrier(0); x = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define K3P_T(x) do { } while (0)
#endif

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
    ld_tile<KS>(a, db, min(t, n_tiles - 1), lane);
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
  // two tile buffers in rotation (a register copy `a = an` would wait for the prefetch)
  auto body = [&](const h16x8(&a)[NP], h16x8(&an)[NP], int t) {
    {  // prefetch the next tile of this wave (clamped: always issue, never branch per load)
      ld_tile<KS>(an, db, min(t + NW, n_tiles - 1), lane);
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
  };
  for (; t < t_end; t += 2 * NW) {
    body(a, an, t);
    if (t + NW >= t_end) break;
    body(an, a, t + NW);
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

// ------------------------------------------------------------------------------------------
// K3p: the certified pruned scan (1 channel).  The level's DB is Morton-sorted
// in the projection space of its top IA_NPC principal axes (ia_prune.hip: position -> row table
// pos2row, per-tile projection boxes); K2p wrote each query's projection interval, bound U' and
// key (ia_prune.h).  Per workgroup:
//   1. rank-sort the step's queries by key in LDS (deterministic: ties by query index) and
//      gather this launch's QT query tiles in sorted order, so a query tile is compact in
//      projection space too; per query tile a bounding box of its intervals and max U'
//   2. DB tiles round-robin: WG w, wave v takes tiles w + nwg*(v + NW*k) (the merge rescans the
//      same chunk, MergeArgs::rr); per tile a need mask over the query tiles: a coarse
//      tile-box test (lanes = query tiles), then for the survivors the per-query test
//      LB(q, tile) <= U'_q (lanes = queries, ballot).  Tiles nobody needs are never loaded; the
//      next needed tile is prefetched while the current one is contracted
//   3. only the needed (DB tile, query tile) pairs run the 12-MFMA chain (two chains at once
//      when both tiles of a query-tile pair are needed) with the packed-index epilogue
//   4. per-query records as K3h, written to the queries' original slots with DB rows taken
//      from pos2row; the WG adds its computed pair count to *pairs (flop accounting)
// Skipped rows are strictly farther than the query's coherence candidate (ia_prune.h), so
// they can neither be nor tie the exact NN; K4's certification over the computed rows stands.
// ------------------------------------------------------------------------------------------
template <int KS>
__device__ __forceinline__ f32x16 k3p_chain(const h16x8 (&a)[2 * KS], const h16x8 *qb) {
  f32x16 c = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; s++) {
    const h16x8 xh = qb[(2 * s) * IA_WAVE], xl = qb[(2 * s + 1) * IA_WAVE];
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s + 1], xh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], xl, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], xh, c, 0, 0, 0);
  }
  return c;
}
template <int KS>
__device__ __forceinline__ void k3p_chain2(const h16x8 (&a)[2 * KS], const h16x8 *qb0, const h16x8 *qb1, f32x16 &c0,
                                           f32x16 &c1) {
  constexpr f32x16 zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  c0 = zero;
  c1 = zero;
#pragma unroll
  for (int s = 0; s < KS; s++) {
    const h16x8 x0h = qb0[(2 * s) * IA_WAVE], x0l = qb0[(2 * s + 1) * IA_WAVE];
    const h16x8 x1h = qb1[(2 * s) * IA_WAVE], x1l = qb1[(2 * s + 1) * IA_WAVE];
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s + 1], x0h, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s + 1], x1h, c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], x0l, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], x1l, c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], x0h, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], x1h, c1, 0, 0, 0);
  }
}
// packed epilogue of one accumulator into one query's (b1, b2, tile)
__device__ __forceinline__ void k3p_epi1(const f32x16 &e, int t, float &b1, float &b2, int &i1) {
  const float o = b1;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const float p = k3h_pack(e[r], r);
    b2 = k3h_med3(b1, b2, p);
    b1 = k3h_min(b1, p);
  }
  i1 = b1 != o ? t : i1;
}
// query-tile pairs QP.. of one DB tile t; m2 = the pair's two need bits (wave-uniform).  A pair
// with one needed tile runs one chain on it; its query state is selected with v_cndmask (never
// a dynamically indexed register array, which would live in scratch)
template <int KS, int QT, int QP>
__device__ __forceinline__ void k3p_pairs(const h16x8 (&a)[2 * KS], const h16x8 *lq, unsigned msk, int t, float (&b1)[QT],
                                          float (&b2)[QT], int (&i1)[QT]) {
  if constexpr (2 * QP < QT) {
    constexpr int NP = 2 * KS, q0 = 2 * QP, q1 = 2 * QP + 1;
    const unsigned m2 = (msk >> q0) & 3u;
    const h16x8 *qb0 = lq + q0 * NP * IA_WAVE;
    if constexpr (q1 < QT) {
      if (m2 == 3u) {
        f32x16 c0, c1;
        k3p_chain2<KS>(a, qb0, qb0 + NP * IA_WAVE, c0, c1);
        k3h_epi2<QT, true>(c0, c1, q0, true, 0, t, b1, b2, i1);
      } else if (m2 != 0u) {
        const bool sel = m2 == 2u;
        const f32x16 c = k3p_chain<KS>(a, sel ? qb0 + NP * IA_WAVE : qb0);
        float x1 = sel ? b1[q1] : b1[q0], x2 = sel ? b2[q1] : b2[q0];
        int xi = sel ? i1[q1] : i1[q0];
        k3p_epi1(c, t, x1, x2, xi);
        b1[q0] = sel ? b1[q0] : x1;
        b2[q0] = sel ? b2[q0] : x2;
        i1[q0] = sel ? i1[q0] : xi;
        b1[q1] = sel ? x1 : b1[q1];
        b2[q1] = sel ? x2 : b2[q1];
        i1[q1] = sel ? xi : i1[q1];
      }
    } else {
      if (m2 == 1u) {
        const f32x16 c = k3p_chain<KS>(a, qb0);
        k3p_epi1(c, t, b1[q0], b2[q0], i1[q0]);
      }
    }
    k3p_pairs<KS, QT, QP + 1>(a, lq, msk, t, b1, b2, i1);
  }
}

// HHF (k3p_variant 14 / 15): each needed (DB tile, query tile) block first runs the hi x hi
// product alone (4 MFMAs); its full product (12 MFMAs) and the top-2 epilogue follow only when
// some value of the block can lie within its query's bound:
//     c_hh <= lim_q = z_q + R_t (w_q + R_t 2^-9 + 2^-20)
// where R_t >= max |a'| over the tile's rows and (z_q, w_q) come from K2p (ia_kernels.hip):
// z_q >= U'_q - |q'|^2 + (rounding terms), w_q >= 2^-8 |q'|.  The hi-only value misses
// sum(hi_a lo_q + lo_a hi_q + lo_a lo_q) and carries its fp32 accumulation error, together
// < 2^-10 (|a'|^2 + 2|a'||q'|) + 2^-24 (16|a'| + 16|q'| + 300) (f16 rounding 2^-11 relative,
// subnormal spacing 2^-25); lim_q takes twice the relative term.  A block that
// fails the test holds only rows with |a - q|^2 > U'_q: they can neither be nor tie the NN, exactly
// like the rows of a tile the box test skips, so the records stay certified.
template <int KS>
__device__ __forceinline__ f32x16 k3p_hh(const h16x8 (&a)[2 * KS], const h16x8 *qb) {
  f32x16 c = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; s++) c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], qb[(2 * s) * IA_WAVE], c, 0, 0, 0);
  return c;
}
// (this file is built with -fno-honor-nans - no value here is ever NaN - so fminf / fmaxf are
// single v_min3 / v_max3 instructions instead of a canonicalizing v_max_f32 x, x per operand
// first; the MFMA read hazards stay the compiler's)
__device__ __forceinline__ float k3p_min16(const f32x16 &c) {
  const float m0 = fminf(fminf(c[0], c[1]), c[2]), m1 = fminf(fminf(c[3], c[4]), c[5]);
  const float m2 = fminf(fminf(c[6], c[7]), c[8]), m3 = fminf(fminf(c[9], c[10]), c[11]);
  const float m4 = fminf(fminf(c[12], c[13]), c[14]);
  return fminf(fminf(fminf(m0, m1), fminf(m2, m3)), fminf(m4, c[15]));
}
// HHX = 3 (k3p_variant 22 / 23): the same filter on a hi-only tile buffer (ld_hi); the blocks
// that pass run their full chains one tile later, from the whole tile loaded only then
template <int KS, int QT, int Q>
__device__ __forceinline__ void k3p_hhpipe_h(const h16x8 (&h)[KS], const h16x8 *lq, unsigned msk, float rt,
                                             const float *qzt, const float *qzw, f32x16 (&acc)[2], unsigned &pass) {
  if constexpr (Q <= QT) {
    constexpr int NP = 2 * KS, QS = NP, PS = 2;
    if constexpr (Q < QT) {
      if ((msk >> Q) & 1u) {
        const h16x8 *qb = lq + Q * QS * IA_WAVE;
        f32x16 c = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        h16x8 qv[KS];  // the block's query pieces, all requested before the first product
#pragma unroll
        for (int s = 0; s < KS; s++) qv[s] = qb[(PS * s) * IA_WAVE];
#pragma unroll
        for (int s = 0; s < KS; s++) c = __builtin_amdgcn_mfma_f32_32x32x16_f16(h[s], qv[s], c, 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, KS, 0);  // the KS LDS reads first (one wait),
        __builtin_amdgcn_sched_group_barrier(0x008, KS, 0);  // then the KS products
        acc[Q & 1] = c;
      }
    }
    if constexpr (Q >= 1) {
      if ((msk >> (Q - 1)) & 1u) {
        const float lim = fmaf(rt, qzw[(Q - 1) * IA_TILE] + fmaf(rt, 0x1p-9f, 0x1p-20f), qzt[(Q - 1) * IA_TILE]);
        pass |= __ballot(k3p_min16(acc[(Q - 1) & 1]) <= lim) != 0ull ? 1u << (Q - 1) : 0u;
      }
    }
    k3p_hhpipe_h<KS, QT, Q + 1>(h, lq, msk, rt, qzt, qzw, acc, pass);
  }
}
// k3p_variant 24 / 25: the same filter walking only the set bits of the need mask (a tile has
// ≈ 2.7 of 11 blocks needed: the unrolled form spends its scalar instructions testing the other
// bits).  Blocks in bit order, two accumulators: a block's products are issued before the
// previous block's bound test, as in k3p_hhpipe_h; the query hi pieces at lq ([QT][KS][64]).
template <int KS>
__device__ __forceinline__ unsigned k3p_filter_bits(const h16x8 (&h)[KS], const h16x8 *lq, unsigned msk, float rt,
                                                    const float *qzt, const float *qzw) {
  const float rr = fmaf(rt, 0x1p-9f, 0x1p-20f);
  auto prod = [&](int q) {
    const h16x8 *qb = lq + q * KS * IA_WAVE;
    f32x16 c = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    h16x8 qv[KS];
#pragma unroll
    for (int s = 0; s < KS; s++) qv[s] = qb[s * IA_WAVE];
#pragma unroll
    for (int s = 0; s < KS; s++) c = __builtin_amdgcn_mfma_f32_32x32x16_f16(h[s], qv[s], c, 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, KS, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, KS, 0);
    return c;
  };
  auto test = [&](const f32x16 &c, int q) -> unsigned {
    const float lim = fmaf(rt, qzw[q * IA_TILE] + rr, qzt[q * IA_TILE]);
    return __ballot(k3p_min16(c) <= lim) != 0ull ? 1u << q : 0u;
  };
  unsigned pass = 0;
  f32x16 a0, a1;
  // a1 is read only after a product wrote it; without a definition here the compiler zeroes its
  // 16 registers at every tile (an empty asm output: no instruction, no hazard - it is never an
  // MFMA result that an asm statement reads)
  asm volatile("" : "=v"(a1));
  int qa = -1, qb = -1;  // the block whose products sit in a0 / a1, its test still due
  for (;;) {
    if (!msk) break;
    qa = __builtin_ctz(msk);
    msk &= msk - 1;
    a0 = prod(qa);
    if (qb >= 0) pass |= test(a1, qb);
    qb = -1;
    if (!msk) break;
    qb = __builtin_ctz(msk);
    msk &= msk - 1;
    a1 = prod(qb);
    pass |= test(a0, qa);
    qa = -1;
  }
  if (qa >= 0) pass |= test(a0, qa);
  if (qb >= 0) pass |= test(a1, qb);
  return pass;
}

// k3p_variant 24 / 25, second pass: the full 12-MFMA chains of a tile's filter-passing blocks
// with the query hi pieces at qh ([QT][KS][64], LDS) and the lo pieces at ql (same layout, LDS):
// the products and their order are k3p_chain's / k3p_chain2's, so values and records are v14's
template <int KS>
__device__ __forceinline__ f32x16 k3p_chain_hl(const h16x8 (&a)[2 * KS], const h16x8 *qh, const h16x8 *ql) {
  f32x16 c = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; s++) {
    const h16x8 xh = qh[s * IA_WAVE], xl = ql[s * IA_WAVE];
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s + 1], xh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], xl, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], xh, c, 0, 0, 0);
  }
  return c;
}
template <int KS>
__device__ __forceinline__ void k3p_chain2_hl(const h16x8 (&a)[2 * KS], const h16x8 *qh0, const h16x8 *ql0, const h16x8 *qh1,
                                              const h16x8 *ql1, f32x16 &c0, f32x16 &c1) {
  constexpr f32x16 zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  c0 = zero;
  c1 = zero;
#pragma unroll
  for (int s = 0; s < KS; s++) {
    const h16x8 x0h = qh0[s * IA_WAVE], x0l = ql0[s * IA_WAVE], x1h = qh1[s * IA_WAVE], x1l = ql1[s * IA_WAVE];
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s + 1], x0h, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s + 1], x1h, c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], x0l, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], x1l, c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], x0h, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], x1h, c1, 0, 0, 0);
  }
}
// k3p_pairs with the query hi / lo pieces in separate LDS arrays (qh, ql: [QT][KS][64], lane offset
// included)
template <int KS, int QT, int QP>
__device__ __forceinline__ void k3p_pairs_hl(const h16x8 (&a)[2 * KS], const h16x8 *qh, const h16x8 *ql, unsigned msk, int t,
                                             float (&b1)[QT], float (&b2)[QT], int (&i1)[QT]) {
  if constexpr (2 * QP < QT) {
    constexpr int QS = KS * IA_WAVE, q0 = 2 * QP, q1 = 2 * QP + 1;
    const unsigned m2 = (msk >> q0) & 3u;
    if constexpr (q1 < QT) {
      if (m2 == 3u) {
        f32x16 c0, c1;
        k3p_chain2_hl<KS>(a, qh + q0 * QS, ql + q0 * QS, qh + q1 * QS, ql + q1 * QS, c0, c1);
        k3h_epi2<QT, true>(c0, c1, q0, true, 0, t, b1, b2, i1);
      } else if (m2 != 0u) {
        const bool sel = m2 == 2u;
        const int qq = sel ? q1 : q0;
        const f32x16 c = k3p_chain_hl<KS>(a, qh + qq * QS, ql + qq * QS);
        float x1 = sel ? b1[q1] : b1[q0], x2 = sel ? b2[q1] : b2[q0];
        int xi = sel ? i1[q1] : i1[q0];
        k3p_epi1(c, t, x1, x2, xi);
        b1[q0] = sel ? b1[q0] : x1;
        b2[q0] = sel ? b2[q0] : x2;
        i1[q0] = sel ? i1[q0] : xi;
        b1[q1] = sel ? x1 : b1[q1];
        b2[q1] = sel ? x2 : b2[q1];
        i1[q1] = sel ? xi : i1[q1];
      }
    } else {
      if (m2 == 1u) {
        const f32x16 c = k3p_chain_hl<KS>(a, qh + q0 * QS, ql + q0 * QS);
        k3p_epi1(c, t, b1[q0], b2[q0], i1[q0]);
      }
    }
    k3p_pairs_hl<KS, QT, QP + 1>(a, qh, ql, msk, t, b1, b2, i1);
  }
}

// HHX paired (k3p_variant 20 / 21): the same fused corrections, organised like k3p_pairs - the
// hi x hi chains of a query-tile pair run as two independent chains, both bound tests follow,
// and the passing blocks' corrections run as two chains (both pass) or one, with the two-query
// epilogue when both pass.  Two independent MFMA chains per pair instead of k3p_hhfuse's
// software pipeline over single chains.
template <int KS>
__device__ __forceinline__ void k3p_corr(const h16x8 (&a)[2 * KS], const h16x8 *qb, f32x16 &c) {
#pragma unroll
  for (int s = 0; s < KS; s++) {
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s + 1], qb[(2 * s) * IA_WAVE], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], qb[(2 * s + 1) * IA_WAVE], c, 0, 0, 0);
  }
}
template <int KS, int QT, int QP>
__device__ __forceinline__ void k3p_hhpairs(const h16x8 (&a)[2 * KS], const h16x8 *lq, unsigned msk, float rt,
                                            const float *qzt, const float *qzw, int t, float (&b1)[QT], float (&b2)[QT],
                                            int (&i1)[QT], unsigned &pass) {
  if constexpr (2 * QP < QT) {
    constexpr int NP = 2 * KS, q0 = 2 * QP, q1 = 2 * QP + 1;
    const unsigned m2 = (msk >> q0) & 3u;
    const h16x8 *qb0 = lq + q0 * NP * IA_WAVE, *qb1 = qb0 + NP * IA_WAVE;
    const float rr = fmaf(rt, 0x1p-9f, 0x1p-20f);
    if constexpr (q1 < QT) {
      if (m2 == 3u) {
        constexpr f32x16 zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        f32x16 c0 = zero, c1 = zero;
#pragma unroll
        for (int s = 0; s < KS; s++) {
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], qb0[(2 * s) * IA_WAVE], c0, 0, 0, 0);
          c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], qb1[(2 * s) * IA_WAVE], c1, 0, 0, 0);
        }
        const bool p0 = __ballot(k3p_min16(c0) <= fmaf(rt, qzw[q0 * IA_TILE] + rr, qzt[q0 * IA_TILE])) != 0ull;
        const bool p1 = __ballot(k3p_min16(c1) <= fmaf(rt, qzw[q1 * IA_TILE] + rr, qzt[q1 * IA_TILE])) != 0ull;
        pass |= (p0 ? 1u << q0 : 0u) | (p1 ? 1u << q1 : 0u);
        if (p0 && p1) {
#pragma unroll
          for (int s = 0; s < KS; s++) {
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s + 1], qb0[(2 * s) * IA_WAVE], c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s + 1], qb1[(2 * s) * IA_WAVE], c1, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], qb0[(2 * s + 1) * IA_WAVE], c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * s], qb1[(2 * s + 1) * IA_WAVE], c1, 0, 0, 0);
          }
          k3h_epi2<QT, true>(c0, c1, q0, true, 0, t, b1, b2, i1);
        } else if (p0) {
          k3p_corr<KS>(a, qb0, c0);
          k3p_epi1(c0, t, b1[q0], b2[q0], i1[q0]);
        } else if (p1) {
          k3p_corr<KS>(a, qb1, c1);
          k3p_epi1(c1, t, b1[q1], b2[q1], i1[q1]);
        }
      } else if (m2 != 0u) {
        const bool sel = m2 == 2u;
        const h16x8 *qb = sel ? qb1 : qb0;
        f32x16 c = k3p_hh<KS>(a, qb);
        const int qq = sel ? q1 : q0;
        if (__ballot(k3p_min16(c) <= fmaf(rt, qzw[qq * IA_TILE] + rr, qzt[qq * IA_TILE])) != 0ull) {
          pass |= 1u << qq;
          k3p_corr<KS>(a, qb, c);
          float x1 = sel ? b1[q1] : b1[q0], x2 = sel ? b2[q1] : b2[q0];
          int xi = sel ? i1[q1] : i1[q0];
          k3p_epi1(c, t, x1, x2, xi);
          b1[q0] = sel ? b1[q0] : x1;
          b2[q0] = sel ? b2[q0] : x2;
          i1[q0] = sel ? i1[q0] : xi;
          b1[q1] = sel ? x1 : b1[q1];
          b2[q1] = sel ? x2 : b2[q1];
          i1[q1] = sel ? xi : i1[q1];
        }
      }
    } else {
      if (m2 == 1u) {
        f32x16 c = k3p_hh<KS>(a, qb0);
        if (__ballot(k3p_min16(c) <= fmaf(rt, qzw[q0 * IA_TILE] + rr, qzt[q0 * IA_TILE])) != 0ull) {
          pass |= 1u << q0;
          k3p_corr<KS>(a, qb0, c);
          k3p_epi1(c, t, b1[q0], b2[q0], i1[q0]);
        }
      }
    }
    k3p_hhpairs<KS, QT, QP + 1>(a, lq, msk, rt, qzt, qzw, t, b1, b2, i1, pass);
  }
}

#if defined(IA_K3H_KS) && defined(IA_K3H_QT)
#define IA_K3H_CAT2(a, b, c) a##b##_##c
#define IA_K3H_CAT(a, b, c) IA_K3H_CAT2(a, b, c)
// variant (option "k3_variant"): 0 = compare/select epilogue, 1 = packed-index epilogue
// The product library holds only the packed-index epilogue (variant 1); the compare/select
// epilogue (0) and the probes (2, 3) are in git history.
k3h_fn IA_K3H_CAT(ia_k3h_get_, IA_K3H_KS, IA_K3H_QT)(int variant) {
  (void)variant;
  return k3h_scan<IA_K3H_KS, IA_K3H_QT, IA_WGH / IA_WAVE, true>;
}
#endif

// ------------------------------------------------------------------------------------------
// K3p (k3p_variants 7, 11, 14, 15, 18..21).  Same pairs, same records semantics
// as V1, organised so no phase waits on another's memory latency:
//   1. ONE global round: every query's pruning record (thread = query, registers), the step's
//      unsorted split-f16 query fragments (coalesced, registers), the workgroup's tile boxes
//      (to LDS) and each wave's speculative first DB tile (PRE: this launch's presorted slice
//      straight into LDS)
//   2. bitonic sort by unique key; fragments and records scattered to their sorted LDS slots;
//      query-tile boxes by 32-lane butterflies (PRE: skipped, or only the boxes)
//   3. tiles handed out through an LDS counter; per tile the coarse (query-tile box) and fine
//      (per query) need tests, the needed tile's load in flight while the previous one is
//      contracted (two register buffers in rotation)
//   4. per-query records exactly as V1
// (The other versions of DESIGN.md §4b's progression - no interleaving, one or three tile
// buffers, software-pipelined single chains, the previous step's order, the rotated-DB head
// filter - are in the history of this file up to round 3.)
// ------------------------------------------------------------------------------------------
#define IA_K3P3_MAXQ 512   // queries per step (one per thread)
// steps of up to IA_K3P_RANK_MAX queries are sorted by rank counting, wider ones by the bitonic
// network (at 342 queries the network measured faster: profiles/r02/ab3, again in round 5:
// profiles/r05/rank_sort)
#define IA_K3P_RANK_MAX 256
// PRE (k3p_variant 11, any Mpad <= 4096): the step's queries were sorted once by k_query_sort
// (ia_prune.hip): qf / qinfo hold them in sorted order (fragments; lo, hi, (U', key) per slot),
// ord_in maps a sorted slot to its query and tbox holds the sorted query tiles' boxes, so phase
// 1 loads only this launch's slice and phase 2 (sort, scatter, tile boxes) is skipped.
// HHF (k3p_variant 14 / 15): the hi x hi block filter above (k3p_hhpipe); the per-WG pair
// counter slot then holds (pairs with corrections << 32) + box-needed pairs.  HHX: how the
// correction products follow the filter (0: full chains, 1: fused single chains, 2: fused on
// query-tile pairs, k3p_hhpairs).
template <int KS, int QT, int NW, bool PRE = false, bool HHF = false, int HHX = 0>
__global__ void __launch_bounds__(NW * IA_WAVE, 1)
k3h_prune3(const h16x8 *__restrict__ db, const h16x8 *__restrict__ qf, const float4 *__restrict__ qinfo,
           const float4 *__restrict__ boxes, const int *__restrict__ pos2row, int NT, int qt0, int M, int Mpad, int nwg,
           float4 *__restrict__ rec, float *__restrict__ recT, unsigned long long *__restrict__ pairs,
           unsigned long long *__restrict__ tiles, int rev, const int *__restrict__ ord_in, int n_in,
           int r0, int *__restrict__ ord_out, const float4 *__restrict__ tbox, const float *__restrict__ tnorm,
           int nqb, int qt_end, XOScan xo) {
  constexpr int NP = 2 * KS, NPAIR = (QT + 1) / 2, WGT = NW * IA_WAVE, NQ = QT * IA_TILE;
  // unsorted fragments per thread (HHX 4: the hi pieces only)
  constexpr int NE = PRE ? 1 : (IA_K3P3_MAXQ / IA_TILE * (HHX == 4 ? KS : NP) * IA_WAVE + WGT - 1) / WGT;
  static_assert(QT <= 32 && 2 * NW >= QT, "need masks are 32-bit; one query tile per half wave");
  // the in-kernel sort holds one query per thread; the tile walk takes any K (the launcher keeps
  // K <= IA_K3P_MAXK_LDS: the boxes, need masks and R_t of the WG's tiles live in LDS)
  static_assert(WGT >= IA_K3P3_MAXQ, "one query per thread");
  static_assert(HHF && HHX >= 2 && HHX <= 4, "the product variants: 20 / 21 (HHX 2), 22 (3), 24 / 25 (4)");
  extern __shared__ h16x8 ldsh[];  // sorted query fragments [QT][NP][64], reused for the merge
  // HHX 4: ldsh holds the hi pieces only ([QT][KS][64]); the waves' LDS-DMA rings of the hi
  // stream ([NW][3] slots of 3.5 KiB; the lo pieces in the second pass) are a static array of
  // their own, so the compiler can tell that no other LDS access aliases a pending DMA (it puts
  // a vmcnt(0) before any LDS access it cannot prove disjoint from one)
  constexpr int QFP = HHX == 4 ? KS : NP;
  __shared__ h16x8 ring[HHX == 4 ? NW * 3 * IA_HSLOT : 1];
  float4 *qlo = reinterpret_cast<float4 *>(ldsh + QT * QFP * IA_WAVE);  // [NQ]
  float4 *qhi = qlo + NQ;                                               // [NQ]
  float *qU = reinterpret_cast<float *>(qhi + NQ);                     // [NQ]
  float4 *tlo = reinterpret_cast<float4 *>(qU + NQ);                   // [QT] query-tile boxes
  float4 *thi = tlo + QT;                                               // [QT]
  float *tU = reinterpret_cast<float *>(thi + QT);                     // [QT]
  unsigned *skey = reinterpret_cast<unsigned *>(tU + ((QT + 3) & ~3));  // [Mpad]   (PRE: [NQ] slice order)
  int *order = reinterpret_cast<int *>(skey + (PRE ? NQ : Mpad));       // [Mpad] sorted -> query
  int *rankof = order + (PRE ? 0 : Mpad);                               // [Mpad] query -> sorted
  // PRE launches may cover several query blocks (nqb > 1): a grid of nqb x nwg workgroups, block
  // b = the presorted query tiles [qt0 + b QT, min(qt0 + (b + 1) QT, qt_end)) against the DB
  // chunk wg (tiles wg + nwg k), so one launch streams the DB once per block instead of one
  // launch per block paying the setup and tail again.  When nwg is a multiple of 8 the blocks of
  // one chunk get workgroup ids equal mod 8, i.e. the same XCD (round-robin dispatch): they read
  // the same tiles at about the same time through one L2.
  int wg = blockIdx.x, qblk = 0;
  if ((PRE || xo.on) && nqb > 1) {
    if ((nwg & 7) == 0) {
      const int grp = wg / (8 * nqb), r = wg - grp * 8 * nqb;
      qblk = r >> 3;
      wg = grp * 8 + (r & 7);
    } else {
      qblk = wg / nwg;
      wg -= qblk * nwg;
    }
    if (PRE) qt0 += qblk * QT;
  }
  if (!PRE && xo.on) {  // owner-computes, in-kernel sort: block qblk = owner qblk's Mpad queries
    qf += (int64_t)qblk * (Mpad / IA_TILE) * NP * IA_WAVE;
    qinfo += 3 * (int64_t)qblk * Mpad;
  }
  const int qtb = PRE ? min(QT, qt_end - qt0) : QT;  // query tiles of this block (PRE: the last may hold fewer)
  const int K = (NT - wg + nwg - 1) / nwg;  // tiles wg + nwg*k, k < K (host: nwg <= NT, K <= IA_K3P_MAXK_LDS)
  // rev: this step walks the workgroup's tiles in reverse (alternate steps: the tiles read last
  // by one step are read first by the next, while they are still in the memory-side cache)
  auto tk = [&](int k) { return wg + nwg * (rev ? K - 1 - k : k); };
  float4 *wbox = reinterpret_cast<float4 *>(rankof + (PRE ? 0 : Mpad));  // [2K] the WG's tile boxes
  unsigned *kmask = reinterpret_cast<unsigned *>(wbox + 2 * K);        // [K] need mask per tile
  int *items = reinterpret_cast<int *>(kmask + K);                     // [K] needed tiles, in order
  float *qzt = reinterpret_cast<float *>(items + K);                    // HHF: [NQ] z per sorted slot
  float *qzw = qzt + NQ;                                                // HHF: [NQ] w per sorted slot
  float *wR = qzw + NQ;                                                 // HHF: [K] R_t of the WG's tiles
  int *plk = reinterpret_cast<int *>(wR + K);                           // HHX 4: [K] filter-passing tiles
  unsigned *plm = reinterpret_cast<unsigned *>(plk + K);                // HHX 4: [K] their passing blocks
  __shared__ unsigned wpairs[NW], wtiles[NW], wfull[NW], wtp[NW];
  __shared__ int pcount, pctr;  // HHX 4: passing tiles listed / handed out
  const int tid = threadIdx.x, lane = tid & 63, half = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int s0 = qt0 * IA_TILE;
  [[maybe_unused]] unsigned long long ph[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  K3P_T(ph[0]);
  const unsigned long long stamp0 = xo.stamp ? ia_clock() : 0ull;

  // ---- 1. one global round
  h16x8 a[NP], an[NP];
  // HHX 4: the wave's first two tiles (static: wave, wave + NW) go to its ring speculatively (93 %
  // of the tiles are needed at 1024^2) once the global round's loads are in, so they are in
  // flight during the query sort (spec_hi below)
  h16x8 *wring = ring + wave * 3 * IA_HSLOT;
  if constexpr (HHX != 4) ld_tile<KS>(a, db, tk(min(wave, K - 1)), lane);
  if constexpr (PRE) {
    if (xo.on) {
      // owner-computes sharded step: this block's tiles come from their owner's K2s (another
      // rank); wait for each tile's flag (bounded: a late peer sets xo.err, never a hang)
      // (after any earlier timeout of this context every wait is skipped: a lost peer costs one
      // timeout, then the level runs to its end and reports IA_ECOMM)
      if (tid < qtb && __hip_atomic_load(xo.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        // relaxed: the area is uncached (no stale line to invalidate); the loads below issue
        // after the barrier, i.e. after every flag was seen
        while (__hip_atomic_load(xo.flag + qt0 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != xo.seq) {
          if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > xo.timeout_ticks) {
            atomicOr(xo.err, 4u);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
    }
    // this launch's slice of the presorted queries, straight into LDS
    const h16x8 *qs = qf + (int64_t)qt0 * NP * IA_WAVE;
    if constexpr (HHX == 4) {  // hi pieces only
      for (int e = tid; e < QT * KS * IA_WAVE; e += WGT) {
        const int pq = e >> 6, qt = pq / KS, s2 = pq - qt * KS;
        ldsh[e] = qt < qtb ? qs[(qt * NP + 2 * s2) * IA_WAVE + (e & 63)] : h16x8{};
      }
    } else {
      for (int e = tid; e < QT * NP * IA_WAVE; e += WGT) ldsh[e] = e < qtb * NP * IA_WAVE ? qs[e] : h16x8{};
    }
    for (int x = tid; x < NQ; x += WGT) {
      const int sl = s0 + x;
      const bool ok = sl < Mpad && x < qtb * IA_TILE;  // slots past the block: padding (never contracted)
      qlo[x] = ok ? qinfo[3 * sl] : make_float4(0.f, 0.f, 0.f, 0.f);
      qhi[x] = ok ? qinfo[3 * sl + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 u = ok ? qinfo[3 * sl + 2] : make_float4(-INFINITY, 0.f, -INFINITY, 0.f);
      qU[x] = u.x;
      if constexpr (HHF) {
        qzt[x] = u.z;
        qzw[x] = u.w;
      }
      skey[x] = ok ? ord_in[sl] : 0x7fffffff;  // slot -> query of this slice
    }
    if (tid < QT && tbox) {  // (tbox = nullptr: the boxes are taken from the slice below)
      const bool ok = tid < qtb;
      tlo[tid] = ok ? tbox[3 * (qt0 + tid)] : make_float4(0.f, 0.f, 0.f, 0.f);
      thi[tid] = ok ? tbox[3 * (qt0 + tid) + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
      tU[tid] = ok ? tbox[3 * (qt0 + tid) + 2].x : -INFINITY;
    }
    for (int x = tid; x < K; x += WGT) {  // K may exceed WGT (up to IA_K3P_MAXK_LDS)
      const int t = tk(x);
      wbox[2 * x] = boxes[2 * t];
      wbox[2 * x + 1] = boxes[2 * t + 1];
      if constexpr (HHF) wR[x] = tnorm[t];
    }
  }
  auto spec_hi = [&]() {
    if constexpr (HHX == 4) {
      dma_hi<KS>(db, tk(min(wave, K - 1)), wring, lane);
      dma_hi<KS>(db, tk(min(wave + NW, K - 1)), wring + IA_HSLOT, lane);
    }
  };
  __shared__ int kctr;  // next tile index to hand out
  if (tid == 0) {
    kctr = HHX == 4 ? 2 * NW : NW;  // HHX 4: each wave's first two tiles are static (the speculative DMAs)
    pcount = 0;
    pctr = 0;
  }
  if constexpr (PRE) {
    __syncthreads();
    spec_hi();
  }
  // the query-tile boxes (min lo, max hi, max U' over the tile's real queries) by 32-lane
  // butterflies over the sorted slots in LDS: the in-kernel-sort path, and the presorted path
  // when the step was sorted by its gathers (option "fuse_sort": no k_query_sort, tbox = nullptr)
  auto tile_boxes = [&]() {
    const int j = 2 * wave + half, x = j * IA_TILE + (lane & 31);
    float4 lo = make_float4(INFINITY, INFINITY, INFINITY, INFINITY), hi = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    float u = -INFINITY;
    if (j < QT && qU[x] != -INFINITY) {  // padding slots (U' = -inf) never widen a box
      lo = qlo[x];
      hi = qhi[x];
      u = qU[x];
    }
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      lo.x = fminf(lo.x, xlane_xor_f(lo.x, o));
      lo.y = fminf(lo.y, xlane_xor_f(lo.y, o));
      lo.z = fminf(lo.z, xlane_xor_f(lo.z, o));
      lo.w = fminf(lo.w, xlane_xor_f(lo.w, o));
      hi.x = fmaxf(hi.x, xlane_xor_f(hi.x, o));
      hi.y = fmaxf(hi.y, xlane_xor_f(hi.y, o));
      hi.z = fmaxf(hi.z, xlane_xor_f(hi.z, o));
      hi.w = fmaxf(hi.w, xlane_xor_f(hi.w, o));
      u = fmaxf(u, xlane_xor_f(u, o));
    }
    if ((lane & 31) == 0 && j < QT) {
      tlo[j] = lo;
      thi[j] = hi;
      tU[j] = u;
    }
  };
  if (PRE && !tbox) {
    tile_boxes();
    __syncthreads();
  }
  if constexpr (!PRE) {
  if (xo.on) {  // owner-computes: wait for each of the block's queries (published by its owner's K2p)
    const unsigned *qs = xo.flag + (int64_t)qblk * Mpad;
    if (tid < Mpad && __hip_atomic_load(xo.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
      const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(qs + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != xo.seq) {
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > xo.timeout_ticks) {
          atomicOr(xo.err, 4u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
  }
  float4 mlo = make_float4(0.f, 0.f, 0.f, 0.f), mhi = mlo;
  float mU = -INFINITY, mzt = -INFINITY, mzw = 0.f;
  unsigned mkey = 0xFFFFFFFFu;
  if (!PRE && tid < Mpad) {
    mlo = qinfo[3 * tid];
    mhi = qinfo[3 * tid + 1];
    const float4 u = qinfo[3 * tid + 2];
    mU = u.x;
    mzt = u.z;
    mzw = u.w;
    mkey = (__float_as_uint(u.y) & 0xFFFFF000u) | (unsigned)tid;  // unique (Mpad <= 4096)
  }
  constexpr int NPL = HHX == 4 ? KS : NP;  // pieces per query tile loaded here (HHX 4: hi, 2s)
  const int ne = Mpad / IA_TILE * NPL * IA_WAVE;
  h16x8 qe[NE];
#pragma unroll
  for (int i = 0; i < NE; i++) {
    int e = tid + WGT * i;
    e = e < ne ? e : 0;
    if constexpr (HHX == 4) e = ((e >> 6) / KS * NP + 2 * ((e >> 6) % KS)) * IA_WAVE + (e & 63);
    qe[i] = qf[e];  // unconditional: equal vmcnt on every path
  }
  for (int x = tid; x < K; x += WGT) {
    const int t = tk(x);
    wbox[2 * x] = boxes[2 * t];
    wbox[2 * x + 1] = boxes[2 * t + 1];
    if constexpr (HHF) wR[x] = tnorm[t];
  }
  if (tid < Mpad) {
    skey[tid] = mkey;
    rankof[tid] = -1;
  }
  __syncthreads();
  K3P_T(ph[1]);
  spec_hi();

  // ---- 2. sort, scatter to sorted slots, query-tile boxes
  if (Mpad > IA_K3P_RANK_MAX) {  // (uniform) up to IA_K3P_RANK_MAX queries the rank count
    // bitonic network over the first 512 threads' unique keys (padding: 0xFFFFFFFF, last):
    // exchanges at distance < 64 are lane swaps, the 6 at distance >= 64 go through LDS (the
    // query-fragment area, free until the scatter below)
    unsigned *sx = reinterpret_cast<unsigned *>(ldsh);
    unsigned v = mkey;
#pragma unroll
    for (int kb = 2; kb <= IA_K3P3_MAXQ; kb <<= 1) {
#pragma unroll
      for (int jb = kb >> 1; jb > 0; jb >>= 1) {
        unsigned o;
        if (jb >= IA_WAVE) {
          // two buffers used in turn: a buffer is rewritten two LDS stages later, after every
          // thread passed the barrier that follows its reads, so one barrier per stage
          unsigned *sb = sx + (((kb == 256 && jb == 128) || (kb == 512 && jb != 128)) ? WGT : 0);
          sb[tid] = v;
          __syncthreads();
          o = sb[tid ^ jb];
        } else {
          o = xlane_xor(v, jb);
        }
        const bool keep_min = ((tid & kb) == 0) == ((tid & jb) == 0);
        v = keep_min ? min(v, o) : max(v, o);
      }
    }
    if (tid < Mpad) {
      const int q = (int)(v & 0xFFFu);
      order[tid] = q;
      rankof[q] = tid;
    }
    __syncthreads();
    if (tid < Mpad) {
      const int x = rankof[tid] - s0;
      if (x >= 0 && x < NQ) {
        qlo[x] = mlo;
        qhi[x] = mhi;
        qU[x] = mU;
        if constexpr (HHF) {
          qzt[x] = mzt;
          qzw[x] = mzw;
        }
      }
    }
  } else if (tid < Mpad) {
    int rank = 0;
    for (int j = 0; j < Mpad; j += 4) {
      const uint4 kk = *reinterpret_cast<const uint4 *>(skey + j);
      rank += (int)(kk.x < mkey) + (int)(kk.y < mkey) + (int)(kk.z < mkey) + (int)(kk.w < mkey);
    }
    order[rank] = tid;
    rankof[tid] = rank;
    const int x = rank - s0;
    if (x >= 0 && x < NQ) {
      qlo[x] = mlo;
      qhi[x] = mhi;
      qU[x] = mU;
      if constexpr (HHF) {
        qzt[x] = mzt;
        qzw[x] = mzw;
      }
    }
  }
  [[maybe_unused]] unsigned long long pa = 0, pb = 0, pc = 0;  // (phase probe stamps)
  K3P_T(pa);
  __syncthreads();
  K3P_T(pb);
#pragma unroll
  for (int i = 0; i < NE; i++) {
    const int e = tid + WGT * i;
    if (e < ne) {
      const int L = e & 63, pq = e >> 6, tq = pq / NPL, p = pq - tq * NPL;  // (HHX 4: p = hi piece s)
      const int x = rankof[tq * IA_TILE + (L & 31)] - s0;
      if (x >= 0 && x < NQ) ldsh[((x >> 5) * NPL + p) * IA_WAVE + (L & 32) + (x & 31)] = qe[i];
    }
  }
  K3P_T(pc);
  tile_boxes();
  [[maybe_unused]] unsigned long long pd = 0, pe = 0;
  K3P_T(pd);
  __syncthreads();
  K3P_T(pe);
#if IA_PROBE & 16
  if (lane == 0 && M == Mpad - 10 && wg < 8) {  // the sort phase: network / rank, barrier, scatter,
    atomicAdd(&k3p_prof[16], pa - ph[1]);        // query-tile boxes, barrier
    atomicAdd(&k3p_prof[17], pb - pa);
    atomicAdd(&k3p_prof[18], pc - pb);
    atomicAdd(&k3p_prof[19], pd - pc);
    atomicAdd(&k3p_prof[20], pe - pd);
  }
#endif
  }  // !PRE
  K3P_T(ph[2]);

  float b1[QT], b2[QT];
  int i1[QT];  // tile of b1 (packed epilogue)
#pragma unroll
  for (int q = 0; q < QT; q++) {
    b1[q] = FLT_MAX;
    b2[q] = FLT_MAX;
    i1[q] = 0x7fffffff;
  }
  unsigned cnt = 0, ntl = 0, nfull = 0, ntp = 0;  // ntp: DB tiles with a filter-passing block
  {
    K3P_T(ph[3]);
    // ---- 3'/4'. need tests interleaved with the contraction: wave v walks tiles k = v mod NW;
    // while tile k is contracted, the next needed tile's load is in flight and the need tests
    // after it run on the VALU (two buffers in rotation)
    const bool cl = lane < QT;
    const float4 ctl = cl ? tlo[lane] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 cth = cl ? thi[lane] : ctl;
    const float ctu = cl ? tU[lane] : -INFINITY;
    auto need_k = [&](int k) -> unsigned {
      const float4 blo = wbox[2 * k], bhi = wbox[2 * k + 1];
      const bool cpass = cl && prune_lb(blo, bhi, ctl, cth) <= ctu;
      const unsigned coarse = (unsigned)__ballot(cpass);
      unsigned msk = 0;
#pragma unroll
      for (int pr = 0; pr < NPAIR; pr++) {
        if ((coarse >> (2 * pr)) & 3u) {
          const int jq = 2 * pr + half, x = jq * IA_TILE + (lane & 31);
          bool nd = false;
          if (jq < QT) nd = prune_lb(blo, bhi, qlo[x], qhi[x]) <= qU[x];
          const unsigned long long b = __ballot(nd);
          msk |= (((unsigned)b != 0u ? 1u : 0u) | ((unsigned)(b >> 32) != 0u ? 2u : 0u)) << (2 * pr);
        }
      }
      return msk & coarse;
    };
    // tiles handed out through an LDS counter (balances the waves' pair counts; the records stay
    // exact, only which subset holds which row varies)
    auto grab = [&]() -> int {
      int g = 0;
      if (lane == 0) g = atomicAdd(&kctr, 1);
      return __builtin_amdgcn_readfirstlane(g);
    };
    auto next_k = [&](int k, unsigned &m) -> int {
      for (; k < K; k = grab()) {
        m = need_k(k);
        if (m) return k;
      }
      m = 0;
      return K;
    };
    if constexpr (HHX == 4) {
    // ---- k3p_variant 24 / 25: two passes over the workgroup's tiles.
    // (a) the hi stream: the hi halves (3.5 of 7 KiB per tile at KS = 4) by LDS-DMA into the
    //     wave's ring of three LDS slots, two tiles in flight while the third is filtered: per tile
    //     the hi x hi filter of its box-needed blocks (k3p_hhpipe_h on the slot); a tile with a
    //     passing block goes to a list in LDS.  The loop issues no other vector-memory instruction
    //     (need tests, the tile counter and the list are LDS / VALU work) and exactly four DMAs per
    //     tile (past the last needed tile the same four from the wave's last tile, into the slot
    //     that is never read), so "vmcnt(8)" before a slot is read waits for that slot alone.
    // (b) after a barrier the query lo pieces are staged into the ring area and the listed tiles
    //     are handed out through an LDS counter: whole tiles (two register buffers) and the full
    //     12-MFMA chains of their passing blocks (k3p_pairs_hl: v14's products and records).
    // Tiles: wave w's first two are w and w + NW (the speculative DMAs issued before the query
    // sort), the others come from the workgroup's LDS counter; the passing tiles go to one list
    // (plk / plm, LDS atomic).  The DMAs are inline asm, which the compiler does not track, so it
    // puts no vmcnt(0) before these LDS atomics (it does for the builtin's DMAs).
    // the box need test of a tile with the wave's per-query bounds held in registers (lane L of
    // pair pr: sorted slot (2 pr + L / 32) 32 + L % 32): no LDS round trip per query-tile pair
    float4 pql[NPAIR], pqh[NPAIR];
    float pqu[NPAIR];
#pragma unroll
    for (int pr = 0; pr < NPAIR; pr++) {
      const int jq = 2 * pr + half, x = jq * IA_TILE + (lane & 31);
      const bool ok = jq < QT;
      pql[pr] = ok ? qlo[x] : make_float4(0.f, 0.f, 0.f, 0.f);
      pqh[pr] = ok ? qhi[x] : make_float4(0.f, 0.f, 0.f, 0.f);
      pqu[pr] = ok ? qU[x] : -INFINITY;
    }
    auto need_r = [&](int k) -> unsigned {
      const float4 blo = wbox[2 * k], bhi = wbox[2 * k + 1];
      // (lanes >= QT: ctu = -inf, never passing; no branch around the test)
      const unsigned coarse = (unsigned)__ballot(prune_lb(blo, bhi, ctl, cth) <= ctu);
      unsigned msk = 0;
#pragma unroll
      for (int pr = 0; pr < NPAIR; pr++) {
        if ((coarse >> (2 * pr)) & 3u) {
          const unsigned long long b = __ballot(prune_lb(blo, bhi, pql[pr], pqh[pr]) <= pqu[pr]);
          // (the two 32-lane halves' bits by scalar compares in asm: the compiler turns the C
          // form into a 64-bit VALU compare and a VALU select + readfirstlane)
          unsigned x0, x1;
          asm("s_cmp_lg_u32 %1, 0\n\ts_cselect_b32 %0, 1, 0" : "=s"(x0) : "s"((unsigned)b) : "scc");
          asm("s_cmp_lg_u32 %1, 0\n\ts_cselect_b32 %0, 2, 0" : "=s"(x1) : "s"((unsigned)(b >> 32)) : "scc");
          msk |= (x0 | x1) << (2 * pr);
        }
      }
      return msk & coarse;
    };
    // the query lo pieces of this launch's sorted slots ([QT][KS][64], the hi layout), gathered
    // from the unsorted fragments through the sort (PRE: the presorted slice) into registers now:
    // the loads are in flight during the stream, and its ring area receives them afterwards
    constexpr int NLO = (QT * KS * IA_WAVE + WGT - 1) / WGT;
    h16x8 lo_r[NLO];
#pragma unroll
    for (int i = 0; i < NLO; i++) {
      const int e = tid + WGT * i;
      const int L = e & 63, pq = e >> 6, qt = pq / KS, s2 = pq - qt * KS;
      int64_t src = -1;
      if (e < QT * KS * IA_WAVE) {
        if constexpr (PRE) {
          if (qt < qtb) src = ((int64_t)(qt0 + qt) * NP + 2 * s2 + 1) * IA_WAVE + L;
        } else {
          const int sx = s0 + qt * IA_TILE + (L & 31);
          if (sx < Mpad) {
            const int mq2 = order[sx];
            src = ((int64_t)(mq2 >> 5) * NP + 2 * s2 + 1) * IA_WAVE + (L & 32) + (mq2 & 31);
          }
        }
      }
      lo_r[i] = qf[src >= 0 ? src : 0];
      if (src < 0) lo_r[i] = h16x8{};
    }
    // the wave's first two tiles (wave, wave + NW) were requested speculatively (before the
    // sort); later ones come from the LDS counter (from 2 NW on: the waves' shares balance) and
    // are requested only when needed, the search for the next needed one (need tests, counter)
    // running one tile ahead, while the older two are in flight.  (The DMAs are inline asm, so
    // the compiler puts no vmcnt(0) before the counter's LDS atomic.)
    int np = 0;  // this wave's passing tiles
    int kown = -1;       // its first one (tile, passing blocks)
    unsigned mown = 0u;
    int kc = wave, kq = wave + NW;                     // tiles in slots sl, sl + 1 (>= K: none)
    const int klast = min(wave, K - 1);                 // the dummy DMA's source (L2-hot)
    unsigned mc = kc < K ? need_r(kc) : 0u, mq = kq < K ? need_r(kq) : 0u;
    auto next_needed = [&](unsigned &m) -> int {  // the next needed tile from the counter (>= K: none)
      m = 0u;
      int k = grab();
      for (; k < K; k = grab()) {
        m = need_r(k);
        if (m) break;
      }
      return k;
    };
    unsigned mn;
    int kn = next_needed(mn);
    int sl = 0;  // ring slot of tile kc
    while (kc < K) {
      const bool ok = kn < K;
      dma_hi<KS>(db, tk(ok ? kn : klast), wring + (sl == 0 ? 2 : sl - 1) * IA_HSLOT, lane);
      unsigned m2 = 0u;
      const int k2 = ok ? next_needed(m2) : K;
      ring_wait<8>();  // slot sl landed; the two younger tiles stay in flight
      if (mc) {  // wave-uniform (0: a speculative tile that is not needed)
        h16x8 hc[KS];
        slot_hi(hc, wring + sl * IA_HSLOT, lane);
        const unsigned pass = k3p_filter_bits<KS>(hc, ldsh + lane, mc, wR[kc], qzt + (lane & 31), qzw + (lane & 31));
        cnt += __popc(mc);
        if (pass) {  // wave-uniform
          nfull += __popc(pass);
          ntp++;
          // one list for the workgroup; a wave's first passing tile is marked (bit 31): the wave
          // itself takes it in the second pass, the others go to the pool
          if (lane == 0) {
            const int x = atomicAdd(&pcount, 1);
            plk[x] = kc;
            plm[x] = pass | (np == 0 ? 0x80000000u : 0u);
          }
          if (np == 0) {
            kown = kc;
            mown = pass;
          }
          np++;
        }
      }
      ntl++;
      kc = kq;
      mc = mq;
      kq = kn;
      mq = mn;
      kn = k2;
      mn = m2;
      sl = sl == 2 ? 0 : sl + 1;
    }
    ring_wait<0>();   // the DMAs past the last tile land before the ring area is reused
    [[maybe_unused]] unsigned long long pq0 = 0, pq1 = 0, pq2 = 0, pq3 = 0;
    K3P_T(pq0);
    // second pass.  A wave with passing tiles starts on its own first one, whose whole tile is
    // requested now (in flight during the barriers); the list's unmarked entries form a pool
    // handed out through pctr
    int kcur = kown;
    unsigned mcur = mown;
    if (kcur >= 0) ld_tile<KS>(a, db, tk(kcur), lane);
    __syncthreads();  // every wave's passing tiles are listed, every ring is idle
    K3P_T(pq1);
    const int npass = pcount;
    auto grab2 = [&]() -> int {  // the next unmarked list entry (>= npass: none)
      int g;
      for (;;) {
        g = 0;
        if (lane == 0) g = atomicAdd(&pctr, 1);
        g = __builtin_amdgcn_readfirstlane(g);
        if (g >= npass || !(plm[g] >> 31)) break;
      }
      return g;
    };
    // the query lo pieces into the ring area ([QT][KS][64], the hi layout): this launch's sorted
    // slots (gathered into registers before the stream)
    h16x8 *qlo_f = ring;
#pragma unroll
    for (int i = 0; i < NLO; i++) {
      const int e = tid + WGT * i;
      if (e < QT * KS * IA_WAVE) qlo_f[e] = lo_r[i];
    }
    // the DB rows of the passing tiles' positions, staged by the second pass behind the lo pieces
    // (rowmap[32 k + j] = pos2row of the WG's tile k, position j): the records' row lookups below
    // are then LDS reads instead of dependent global loads
    int *rowmap = reinterpret_cast<int *>(ring + QT * KS * IA_WAVE);
    if (kcur < 0) {  // no passing tile of its own: the first from the pool
      const int j0 = grab2();
      if (j0 < npass) {
        kcur = plk[j0];
        mcur = plm[j0];
        ld_tile<KS>(a, db, tk(kcur), lane);
      }
    }
    __syncthreads();
    K3P_T(pq2);
    auto step4 = [&](const h16x8(&cur)[NP], h16x8(&nxt)[NP]) {
      const int jn = grab2();
      int kn = -1;
      unsigned mn = 0u;
      if (jn < npass) {
        kn = plk[jn];
        mn = plm[jn];
      }
      ld_tile<KS>(nxt, db, tk(kn >= 0 ? kn : kcur), lane);  // unconditional (equal vmcnt)
      const int prow = pos2row[(int64_t)tk(kcur) * IA_TILE + (lane & 31)];
      asm volatile("" ::: "memory");
      k3p_pairs_hl<KS, QT, 0>(cur, ldsh + lane, qlo_f + lane, mcur, kcur, b1, b2, i1);  // i1: the WG-local tile
      if (lane < 32) rowmap[kcur * IA_TILE + lane] = prow;
      kcur = kn;
      mcur = mn;
    };
    while (kcur >= 0) {
      step4(a, an);
      if (kcur < 0) break;
      step4(an, a);
    }
    K3P_T(pq3);
#if IA_PROBE & 16
    if (lane == 0 && M == Mpad - 10 && wg < 8) {  // two-pass phases: stream, barrier, lo staging, chains
      atomicAdd(&k3p_prof[12], pq0 - ph[3]);
      atomicAdd(&k3p_prof[13], pq1 - pq0);
      atomicAdd(&k3p_prof[14], pq2 - pq1);
      atomicAdd(&k3p_prof[15], pq3 - pq2);
    }
#endif
    } else {
    unsigned m;
    int k = next_k(wave, m);
    if constexpr (HHX == 3) {
    // ---- k3p_variant 22 / 23: the DB stream carries only the hi halves (3.5 of 7 KiB per tile
    // at KS = 4).  Per tile: the hi x hi filter of its box-needed blocks on a hi buffer (two in
    // rotation, the next tile's in flight); the tile's lo halves are then loaded only when a
    // block passed (its hi halves copied from the hi buffer; else the same load instructions at
    // one lane-uniform address: equal outstanding loads on every path) and its full chains
    // (k3p_pairs: v14's products and records) run one tile later, while the next tile is
    // filtered.  MALL / HBM bytes: hi of every needed tile + lo of the passing ones (15 % of the
    // loaded tiles at cfg3 with option nn_bound, 46 % without).
    h16x8 ha[KS], hb[KS];
    const int k_spec = min(wave, K - 1);  // the global round's speculative tile, now L2-hot
    ld_hi<KS>(ha, db, tk(k < K ? k : k_spec), lane);
    unsigned pprev = 0u;
    int kprev = 0;
    auto step3 = [&](const h16x8(&cur)[KS], h16x8(&nxt)[KS]) {
      unsigned mn;
      const int kn = next_k(grab(), mn);
      ld_hi<KS>(nxt, db, tk(kn < K ? kn : k), lane);  // unconditional (see below)
      asm volatile("" ::: "memory");  // LDS query fragments are re-read per tile, not hoisted
      f32x16 acc[2];
      unsigned pass = 0;
      k3p_hhpipe_h<KS, QT, 0>(cur, ldsh + lane, m, wR[k], qzt + (lane & 31), qzw + (lane & 31), acc, pass);
      if (pprev) k3p_pairs<KS, QT, 0>(a, ldsh + lane, pprev, tk(kprev), b1, b2, i1);
      {
        // a passing tile: its lo pieces (the hi ones are copied from cur); otherwise the same
        // instructions at one lane-uniform address (one request each, no bytes streamed), so
        // every path keeps the same outstanding loads
        const h16x8 *src = db + (pass ? tk(k) : tk(k_spec)) * TileFmt<KS>::STRIDE;
#pragma unroll
        for (int s2 = 0; s2 < KS; s2++) a[2 * s2 + 1] = src[pass ? TileFmt<KS>::off(2 * s2 + 1, lane) : 0];
        if (pass) {
#pragma unroll
          for (int s2 = 0; s2 < KS; s2++) a[2 * s2] = cur[s2];
        }
      }
      nfull += __popc(pass);
      ntp += pass != 0u;
      pprev = pass;
      kprev = k;
      cnt += __popc(m);
      ntl++;
      k = kn;
      m = mn;
    };
    while (k < K) {
      step3(ha, hb);
      if (k >= K) break;
      step3(hb, ha);
    }
    if (pprev) k3p_pairs<KS, QT, 0>(a, ldsh + lane, pprev, tk(kprev), b1, b2, i1);
    } else {
    // (re)load the first needed tile unconditionally (usually the speculative one again: a
    // cache hit), so the loop is entered with the same outstanding loads on every path
    ld_tile<KS>(a, db, tk(k < K ? k : min(wave, K - 1)), lane);
    auto step = [&](const h16x8(&cur)[NP], h16x8(&nxt)[NP]) {
      unsigned mn;
      const int kn = next_k(grab(), mn);
      // always issue the 8 loads (past the last tile: the current tile again, an L2 hit): with a
      // conditional prefetch the compiler's vmcnt at the join covers the no-load path, which
      // makes the MFMAs below wait for the prefetch itself
      ld_tile<KS>(nxt, db, tk(kn < K ? kn : k), lane);
      asm volatile("" ::: "memory");  // LDS query fragments are re-read per tile, not hoisted
      {  // HHX 2: the fused corrections on query-tile pairs
        unsigned pass = 0;
        k3p_hhpairs<KS, QT, 0>(cur, ldsh + lane, m, wR[k], qzt + (lane & 31), qzw + (lane & 31), tk(k), b1, b2, i1, pass);
        nfull += __popc(pass);
        ntp += pass != 0u;
      }
      cnt += __popc(m);
      ntl++;
      k = kn;
      m = mn;
    };
    while (k < K) {
      step(a, an);
      if (k >= K) break;
      step(an, a);
    }
    }  // HHX != 3
    }  // HHX != 4
  }
  K3P_T(ph[4]);
  if constexpr (HHX == 4) {
    // i1 holds WG-local tiles whose rows the second pass staged in LDS (every wave's)
    const int *rowmap = reinterpret_cast<const int *>(ring + QT * KS * IA_WAVE);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < QT; q++) {
      const int r = (int)(__float_as_uint(b1[q]) & 15u);
      i1[q] = b1[q] == FLT_MAX ? 0x7fffffff : rowmap[i1[q] * IA_TILE + 4 * half + (r & 3) + 8 * (r >> 2)];
    }
  } else {
#pragma unroll
  for (int q = 0; q < QT; q++) {  // tile + packed in-tile index -> DB position (-> DB row)
    const int r = (int)(__float_as_uint(b1[q]) & 15u);
    const int pos = i1[q] * IA_TILE + 4 * half + (r & 3) + 8 * (r >> 2);
    // the lane's candidate rows are looked up here, their loads in flight while the workgroup
    // waits for its slowest wave and merges; the merge then orders ties by row instead of
    // position (any order is exact: K4 reranks the listed rows and T bounds every other one)
    i1[q] = b1[q] == FLT_MAX ? 0x7fffffff : pos2row[pos];
  }
  }  // HHX != 4

  // ---- 5. merge the 2*NW subsets of each query; records go to the original query slots
  // (the slice's query order is read before the reduction area, which extends past the
  // fragments for NW = 16, overwrites it)
  const int mq_pre = tid < NQ ? (PRE ? (int)skey[tid] : order[s0 + tid]) : 0;
  __syncthreads();
  K3P_T(ph[6]);  // probe: the wait for the workgroup's slowest wave ends here
  if (lane == 0) {
    wpairs[wave] = cnt;
    wtiles[wave] = ntl;
    wfull[wave] = nfull;
    wtp[wave] = ntp;
  }
  Top2 *red = reinterpret_cast<Top2 *>(ldsh);  // [NW][QT][32], inside the query-fragment area
  // HHX 4: every lane's subset (b1, b2 as T, row) goes to LDS as it stands
  // ([NW][QT][64] per field) and the per-query merge takes 16 subsets: no half-wave merge
  float *rv1 = reinterpret_cast<float *>(ldsh), *rvT = rv1 + NW * QT * IA_WAVE;
  int *ri1 = reinterpret_cast<int *>(rvT + NW * QT * IA_WAVE);
  constexpr bool T16 = HHX == 4;
  if constexpr (T16) {
#pragma unroll
    for (int q = 0; q < QT; q++) {
      const int ix = (wave * QT + q) * IA_WAVE + lane;
      rv1[ix] = b1[q];
      rvT[ix] = b2[q];
      ri1[ix] = i1[q];
    }
  } else {
#pragma unroll
  for (int q = 0; q < QT; q++) {
    // the two halves of the wave hold the same query's subsets: (b1, row) + runner-up value each;
    // exchanged with v_permlane32_swap, merged with selects (half 0 stores)
    const auto sb = __builtin_amdgcn_permlane32_swap(__float_as_uint(b1[q]), __float_as_uint(b1[q]), false, false);
    const auto si = __builtin_amdgcn_permlane32_swap((unsigned)i1[q], (unsigned)i1[q], false, false);
    const auto s2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(b2[q]), __float_as_uint(b2[q]), false, false);
    const Top2 mine = {b1[q], FLT_MAX, b2[q], i1[q], 0x7fffffff};
    const Top2 other = {__uint_as_float(half ? sb[0] : sb[1]), FLT_MAX, __uint_as_float(half ? s2[0] : s2[1]),
                        (int)(half ? si[0] : si[1]), 0x7fffffff};
    if (half == 0) red[(wave * QT + q) * IA_TILE + lane] = top2_merge_sel(mine, other);
  }
  }  // !T16
  K3P_T(ph[7]);
  __syncthreads();
  K3P_T(ph[8]);
  // (option "rec_wt") buffer descriptors of the record arrays, from kernel arguments only
  const int nrec = M * nwg;
  const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(rec, 0, nrec * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc(recT, 0, nrec * 4, 0x00020000);
  for (int x = tid; x < NQ; x += WGT) {
    Top2 m;
    if constexpr (T16) {
      const int b0 = (x >> 5) * IA_WAVE + (x & 31);  // wave 0, lane x % 32 of query tile x / 32
      // the 2 NW subsets merged as a tree (depth log2(2 NW) instead of a chain of 2 NW - 1; round 6:
      // K3p workgroups 29.4 -> 29.0 us, profiles/r06/tree/): the merge keeps the two
      // lexicographically smallest (value, row) pairs and the smallest other value, which no merge
      // order changes (bit-identical records)
      Top2 t[2 * NW];
#pragma unroll
      for (int e = 0; e < 2 * NW; e++) {
        const int ix = b0 + (e >> 1) * QT * IA_WAVE + (e & 1) * 32;
        t[e] = Top2{rv1[ix], FLT_MAX, rvT[ix], ri1[ix], 0x7fffffff};
      }
#pragma unroll
      for (int st = 1; st < 2 * NW; st <<= 1)
#pragma unroll
        for (int e = 0; e < 2 * NW; e += 2 * st) t[e] = top2_merge_sel(t[e], t[e + st]);
      m = t[0];
    } else {
      m = red[x];
#pragma unroll
      for (int w = 1; w < NW; w++) m = top2_merge_sel(m, red[(w * QT) * IA_TILE + x]);
    }
    const int mq = WGT >= NQ ? mq_pre : (PRE ? (int)skey[x] : order[s0 + x]);
    if (mq < M) {
      const int r1 = m.i1, r2 = m.i2;  // DB rows (looked up before the merge, above)
      const float4 rv = make_float4(m.v1, __int_as_float(r1), m.v2, __int_as_float(r2));
      if (xo.on) {
        // owner-computes sharded step: into the block's owner's area, record w = s nch + wg of
        // sorted slot s0 + x (consecutive x: contiguous stores), then (T, seq) once it is visible
        char *ar = xo.area[qblk / xo.bpj];
        const int64_t slot = (PRE ? 0 : (int64_t)qblk * Mpad) + s0 + x;
        const int64_t ix = ((int64_t)xo.s * nwg + wg) * xo.Mrec + slot;
        if (!PRE && xo.s == qblk && wg == 0) xo.inv[(int64_t)qblk * Mpad + mq] = (int)slot;  // the owner's table
        reinterpret_cast<float4 *>(ar + XOLayout::REC)[ix] = rv;
        ia_stores_done();
        __hip_atomic_store(reinterpret_cast<unsigned long long *>(ar + XOLayout::RTS) + ix,
                           ((unsigned long long)xo.seq << 32) | __float_as_uint(m.T), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      } else if (xo.rec_wt) {
        // option "rec_wt": write-through (sc1) stores, so the kernel boundary finds no partially
        // dirty record lines in this XCD's L2 to write back; the merge reads them
        // after the boundary either way
        const int64_t ix = (int64_t)mq * nwg + wg;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, rv), rrs, (int)(ix * 16), 0, 16);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(m.T), trs, (int)(ix * 4), 0, 16);
      } else {
        rec[(int64_t)mq * nwg + wg] = rv;
        recT[(int64_t)mq * nwg + wg] = m.T;
      }
    }
  }
  K3P_T(ph[9]);
  if (tid == 0) {  // the workgroup's own counter slots (stream-ordered launches: no atomics)
    unsigned long long sp = 0, st = 0, sf = 0, stp = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
      sp += wpairs[w];
      st += wtiles[w];
      sf += wfull[w];
      stp += wtp[w];
    }
    pairs[blockIdx.x] += sp + (HHF ? sf << 32 : 0ull);
    tiles[blockIdx.x] += st + (stp << 32);  // (tiles with a filter-passing block << 32) + tiles loaded
    // DB half-tiles loaded besides one per loaded tile (the algorithmic bytes):
    // whole tiles (HHX <= 2): the lo half of each; hi-only stream (3): the lo halves of the
    // passing tiles; two passes (4): the passing tiles again, whole
    tiles[blockIdx.x + 2 * IA_NWG_H] += HHX == 4 ? 2 * stp : HHX == 3 ? stp : st;
  }
  if (xo.stamp) {  // (uniform) option "stamps": the workgroup's first and last tick
    __syncthreads();
    if (tid == 0) ia_stamp_wg(xo.stamp, stamp0);
  }
#if IA_PROBE & 16
  K3P_T(ph[5]);
  if (lane == 0 && M == Mpad - 10 && wg < 8) {
    atomicAdd(&k3p_prof[0], ph[1] - ph[0]);
    atomicAdd(&k3p_prof[1], ph[2] - ph[1]);
    atomicAdd(&k3p_prof[2], ph[3] - ph[2]);
    atomicAdd(&k3p_prof[3], ph[4] - ph[3]);
    atomicAdd(&k3p_prof[7], ph[5] - ph[4]);
    atomicAdd(&k3p_prof[8], ph[6] - ph[4]);  // the tail's barrier wait
    atomicAdd(&k3p_prof[9], ph[7] - ph[6]);    // per-wave half merge + LDS writes
    atomicAdd(&k3p_prof[10], ph[8] - ph[7]);   // second barrier
    atomicAdd(&k3p_prof[11], ph[9] - ph[8]);   // subset merge + record stores
    atomicAdd(&k3p_prof[4], 1ull);
    atomicAdd(&k3p_prof[5], (unsigned long long)ntl);
    atomicAdd(&k3p_prof[6], (unsigned long long)cnt);
  }
#endif
}

#if (IA_PROBE & 16) && defined(IA_K3H_KS) && defined(IA_K3H_QT) && IA_K3H_KS == 4 && IA_K3H_QT == 11
void ia_k3p_probe_dump() {  // diagnostic build only: phase cycles per plateau wave, to stderr
  unsigned long long v[24];
  if (hipMemcpyFromSymbol(v, HIP_SYMBOL(k3p_prof), sizeof(v)) != hipSuccess || v[4] == 0) return;
  fprintf(stderr, "K3P_PROBE sort phase: network %.0f, barrier %.0f, fragment scatter %.0f, tile boxes %.0f, barrier %.0f\n",
          (double)v[16] / v[4], (double)v[17] / v[4], (double)v[18] / v[4], (double)v[19] / v[4], (double)v[20] / v[4]);
  fprintf(stderr, "K3P_PROBE two-pass (v24/25): stream %.0f, barrier %.0f, lo staging %.0f, chains %.0f\n", (double)v[12] / v[4],
          (double)v[13] / v[4], (double)v[14] / v[4], (double)v[15] / v[4]);
  fprintf(stderr, "K3P_PROBE tail split: half merge %.0f, barrier %.0f, subset merge + records %.0f\n", (double)v[9] / v[4],
          (double)v[10] / v[4], (double)v[11] / v[4]);
  fprintf(stderr, "K3P_PROBE v3 phases if variant>=3: load=setup, sort+scatter=need, need=loop, loop=tail, tail=[7]\n");
  fprintf(stderr, "K3P_PROBE [7]=%.0f [8]=%.0f ([8] = the tail barrier wait)\n", (double)v[7] / v[4],
          (double)v[8] / v[4]);
  fprintf(stderr, "K3P_PROBE waves=%llu setup=%.0f need=%.0f loop=%.0f tail=%.0f tiles/wave=%.2f pairs/wave=%.2f (cycles/wave)\n",
          v[4], (double)v[0] / v[4], (double)v[1] / v[4], (double)v[2] / v[4], (double)v[3] / v[4], (double)v[5] / v[4],
          (double)v[6] / v[4]);
  unsigned long long z[24] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(k3p_prof), z, sizeof(z));
}
#endif

#if defined(IA_K3H_KS) && defined(IA_K3H_QT)
// pruned scan instance (1 channel only: KS = 4)
// The product library holds the pruned scans of DESIGN.md §4b that are still selectable (the
// earlier versions - no filter, single chains, v0-v19 and v23 - are in the history of this
// file up to round 4): in-kernel query sort (steps of <= 512 queries) / presorted form.
k3p_fn IA_K3H_CAT(ia_k3p_get_, IA_K3H_KS, IA_K3H_QT)(int variant) {
  if constexpr (IA_K3H_KS == 4) {
    constexpr int NW = IA_WGH / IA_WAVE;
    // 20 / 21: whole tiles in two register buffers, the fused corrections on query-tile pairs
    if (variant == 20) return k3h_prune3<IA_K3H_KS, IA_K3H_QT, NW, false, true, 2>;
    if (variant == 21) return k3h_prune3<IA_K3H_KS, IA_K3H_QT, NW, true, true, 2>;
    // 22: the filter on hi-only tile loads, full chains of the passing tiles one tile later
    if (variant == 22) return k3h_prune3<IA_K3H_KS, IA_K3H_QT, NW, false, true, 3>;
    // 24 / 25: a hi stream three tiles deep, then the passing tiles' full chains (two passes)
    if (variant == 24) return k3h_prune3<IA_K3H_KS, IA_K3H_QT, NW, false, true, 4>;
    if (variant == 25) return k3h_prune3<IA_K3H_KS, IA_K3H_QT, NW, true, true, 4>;
    return nullptr;
  } else {
    return nullptr;
  }
}
#endif
