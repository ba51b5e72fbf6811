// ia_kernels.hip — CDNA4 (gfx950) kernels of the Image Analogies best-match path.
//
//   K0 k_part_means      deterministic per-(part, channel) means used to centre features
//   K1 k_db_build        create_index's DB rows (algorithms.py:11-47,50-70) -> fp32 MFMA
//                        fragment tiles in HBM (+ row norms, + max row norm R)
//   K2 k_gather_query    BBp_feat of every pixel of one wavefront step
//                        (image_analogies.py:166-168, algorithms.py:78-89) -> fp64 rows +
//                        fp32 fragments staged for K3
//   K3 k3_dist           best_approximate_match's distance scan (algorithms.py:73-75) as a
//                        v_mfma_f32_32x32x2_f32 contraction |a'|^2 - 2 q'.a' with a fused
//                        per-query top-2 + certification threshold kept in registers
//   K4 k_merge_level     exact fp64 rerank of the MFMA candidates (numpy pairwise-sum order,
//                        lowest-index ties), certification with exact fallback rescan,
//                        best_coherence_match (algorithms.py:92-130), compute_distance
//                        (:133-135), the kappa rule (image_analogies.py:206) and the
//                        B'/s/im writeback (:214-220), one wave per query pixel
//   dense variants for the FLANN-compatible index (ia_index_*).
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (no FMA contraction: the exact
// fp64 paths must round exactly like numpy's separate multiply and add).
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include <mutex>
#include <unordered_set>

#include "ia_internal.h"
#include "ia_prune.h"

#ifndef IA_PROBE
#define IA_PROBE 0  // diagnostic phase-stamp builds (8: merge, 16: K3p, 256: K2r; never the product build)
#endif
// waves (= queries) per workgroup of the one-wave-per-query kernels K2h, K2p, K4: one, so a
// step's few hundred latency-bound waves spread over as many CUs (their L1, TA and LDS) as
// possible; 3.35 -> 3.44 M px/s against 4 per workgroup on one box (profiles/r02/wpb)
#ifndef IA_PQ_WPB
#define IA_PQ_WPB 1
#endif
#define IA_PQ_WG (IA_WAVE * IA_PQ_WPB)
#ifndef IA_K4_RPL8
#define IA_K4_RPL8 0  // 1: the fused merge always reads 8 records per lane (A/B builds)
#endif
#if IA_PROBE & 8  // diagnostic build only: s_memtime phase stamps of sampled merge waves
#define IA_STAMP(k) do { __builtin_amdgcn_sched_barrier(0); stamp[k] = __builtin_amdgcn_s_memtime(); \
                         __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define IA_STAMP(k) do { } while (0)
#endif
#if IA_PROBE & 256  // diagnostic build only: s_memtime phase stamps of sampled K2r waves
#define IA_STAMP2(k) do { __builtin_amdgcn_sched_barrier(0); st2[k] = __builtin_amdgcn_s_memtime(); \
                          __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define IA_STAMP2(k) do { } while (0)
#endif


// ------------------------------------------------------------------------------------------
// feature geometry, compile-time per channel count
// ------------------------------------------------------------------------------------------
template <int CH>
struct Geo {
  static constexpr int D = 55 * CH;
  static constexpr int DP = ((D + 1 + 7) / 8) * 8;  // + norm column, 16-B aligned halves
  static constexpr int KH = DP / 2;                 // k-steps of the 32x32x2 chain
  static constexpr int KP = KH / 4;                 // float4 pieces per lane
  static constexpr int DS = ((D + 7) / 8) * 8;      // fp64 row-major DB row stride (doubles)
};

// reflected (symmetric-pad) offsets of the 3x3 coarse and 5x5 fine windows of pixel (r, c)
struct Px {
  int64_t yc[3], yf[5];  // row offsets (already * width * CH)
  int xc[3], xf[5];      // column offsets (already * CH)
};
template <int CH>
__device__ __forceinline__ Px make_px(const Imgs &I, int r, int c) {
  Px P;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    P.yc[k] = (int64_t)ia_reflect((r >> 1) + k - 1, I.hc) * I.wc * CH;
    P.xc[k] = ia_reflect((c >> 1) + k - 1, I.wc) * CH;
  }
#pragma unroll
  for (int k = 0; k < 5; k++) {
    P.yf[k] = (int64_t)ia_reflect(r + k - 2, I.h) * I.w * CH;
    P.xf[k] = ia_reflect(c + k - 2, I.w) * CH;
  }
  return P;
}
// value of feature f (reference order) of pixel P of image `img`
// (A' index; 0 on the B side)
template <int CH>
__device__ __forceinline__ double featp(const Imgs &I, const Px &P, int f, int img) {
  if (f < 9 * CH) {
    const int k = f / CH, ch = f % CH;
    return I.p0[P.yc[k / 3] + P.xc[k % 3] + ch];
  } else if (f < 34 * CH) {
    const int k = (f - 9 * CH) / CH, ch = (f - 9 * CH) % CH;
    return I.p1[P.yf[k / 5] + P.xf[k % 5] + ch];
  } else if (f < 43 * CH) {
    const int k = (f - 34 * CH) / CH, ch = (f - 34 * CH) % CH;
    return I.p2[img * I.img_stride_c + P.yc[k / 3] + P.xc[k % 3] + ch];
  } else {
    const int k = (f - 43 * CH) / CH, ch = (f - 43 * CH) % CH;
    return I.p3[img * I.img_stride_f + P.yf[k / 5] + P.xf[k % 5] + ch];
  }
}
template <int CH>
__device__ __forceinline__ double feat(const Imgs &I, int f, int r, int c, int img) {
  int part, k, ch;
  if (f < 9 * CH) {
    part = 0; k = f / CH; ch = f % CH;
  } else if (f < 34 * CH) {
    part = 1; k = (f - 9 * CH) / CH; ch = (f - 9 * CH) % CH;
  } else if (f < 43 * CH) {
    part = 2; k = (f - 34 * CH) / CH; ch = (f - 34 * CH) % CH;
  } else {
    part = 3; k = (f - 43 * CH) / CH; ch = (f - 43 * CH) % CH;
  }
  if (part == 0 || part == 2) {  // 3x3 at (floor(r/2), floor(c/2)) of the padded coarse level
    int y = ia_reflect((r >> 1) + k / 3 - 1, I.hc), x = ia_reflect((c >> 1) + k % 3 - 1, I.wc);
    const double *b = part == 0 ? I.p0 : I.p2 + img * I.img_stride_c;
    return b[((int64_t)y * I.wc + x) * CH + ch];
  } else {  // 5x5 at (r, c) of the padded fine level (part 3 only reaches k < 12)
    int y = ia_reflect(r + k / 5 - 2, I.h), x = ia_reflect(c + k % 5 - 2, I.w);
    const double *b = part == 1 ? I.p1 : I.p3 + img * I.img_stride_f;
    return b[((int64_t)y * I.w + x) * CH + ch];
  }
}

// the B side of job jp as the four images its query rows read (B-side FeatDesc parts)
__device__ __forceinline__ Imgs job_imgs(Imgs B, const JobPtrs &jp) {
  B.p0 = jp.Bc;
  B.p1 = jp.B;
  B.p2 = jp.Bpc;
  B.p3 = jp.Bp;
  return B;
}

template <int CH>
__device__ __forceinline__ int feat_part(int f) {
  return f < 9 * CH ? 0 : f < 34 * CH ? 1 : f < 43 * CH ? 2 : 3;
}
template <int CH>
__device__ __forceinline__ int feat_ch(int f) {
  return (f < 9 * CH ? f : f < 34 * CH ? f - 9 * CH : f < 43 * CH ? f - 34 * CH : f - 43 * CH) % CH;
}

// numpy pairwise_sum (loops_utils.h.src) over n <= 128 terms produced in order by term(i)
template <int N, class T>
__device__ __forceinline__ double pw_block(T &&term, int off) {
  static_assert(N <= 128, "block");
  if constexpr (N < 8) {
    double res = 0.;
#pragma unroll
    for (int i = 0; i < N; i++) res += term(off + i);
    return res;
  } else {
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] = term(off + j);
    constexpr int NB = N - (N % 8);
#pragma unroll
    for (int i = 8; i < NB; i += 8) {
#pragma unroll
      for (int j = 0; j < 8; j++) r[j] += term(off + i + j);
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (int i = NB; i < N; i++) res += term(off + i);
    return res;
  }
}
// Correctly rounded fp64 square root, as numpy's np.sqrt / np.linalg.norm give on the host.
// Insurance against a device sqrt expansion that is not correctly rounded (the 1-ulp golden
// differences first blamed on it turned out to be libm pow, see pow2_alt): the result is
// settled among sqrt(x) and its two neighbours by the exact residual |x - y*y| (one fused
// multiply-add each).  Nearest-in-square equals nearest-in-root except in a window of relative
// width ~2^-106 around the rounding midpoint.
__device__ __forceinline__ double cr_sqrt(double x) {
  double y = sqrt(x);
  if (!(x > 0.) || !(x < DBL_MAX)) return y;
  const long long b = __double_as_longlong(y);
  const double yl = __longlong_as_double(b - 1), yh = __longlong_as_double(b + 1);
  double r = fabs(__builtin_fma(-y, y, x));
  const double rl = fabs(__builtin_fma(-yl, yl, x)), rh = fabs(__builtin_fma(-yh, yh, x));
  if (rl < r) {
    y = yl;
    r = rl;
  }
  if (rh < r) y = yh;
  return y;
}

// compute_distance's final `** 2` is libm pow(y, 2.0) on a numpy scalar, K4 uses y * y.  They
// differ only when the exact square lies next to a rounding midpoint (glibc pow is accurate to
// ~0.52 ulp; measured: every difference has |y*y - hi| >= 0.986 half-ulp).  pow2_alt returns the
// other value pow may give there (hi itself elsewhere) so K4 can flag a kappa decision that
// would flip between the two (pstat bit 29, ia_stats.kappa_ambiguous).
__device__ __forceinline__ double pow2_alt(double y, double hi) {
  if (!(hi > 0.) || !(hi < DBL_MAX)) return hi;
  const double lo = __builtin_fma(y, y, -hi);  // y*y = hi + lo exactly
  const long long b = __double_as_longlong(hi);
  const double half = 0.5 * (__longlong_as_double(b + 1) - hi);
  if (fabs(lo) < 0.9 * half) return hi;
  return __longlong_as_double(lo > 0. ? b + 1 : b - 1);
}
__device__ __forceinline__ bool kappa_ambiguous(double ya, double da, double yc, double dc, double kf) {
  const double aa = pow2_alt(ya, da), ac = pow2_alt(yc, dc);
  const bool dec = dc <= da * kf;
  if (ya == yc) return (ac <= aa * kf) != dec;  // one value: pow rounds both the same way
  return ((ac <= da * kf) != dec) || ((dc <= aa * kf) != dec) || ((ac <= aa * kf) != dec);
}

// x.x in the summation order of numpy's dot (x.dot(x) inside np.linalg.norm(ord=2), i.e.
// compute_distance, algorithms.py:133-135) on the host that produced the golden vectors: OpenBLAS
// 0.3.29 ddot, SkylakeX kernel (found by matching np.dot bit-for-bit for n = 1..165,
// oracle/ia_oracle.py blas_ddot).  n1 = N & -16 elements go through fused multiply-adds: 32-wide
// blocks into four 8-lane accumulators, whose halves are added into four 4-lane accumulators
// that take any remaining 16-wide block, then ((a0 + a1) + a2) + a3 per lane and
// (l0 + l2) + (l1 + l3); the tail N - n1 elements are fused into the running sum.
template <int N, class X>
__device__ __forceinline__ double blas_dot_sq(X &&x) {
  constexpr int N1 = N & ~15, N32 = N1 & ~31;
  double acc[4][4];
  if constexpr (N32 > 0) {
    double z[4][8];
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int l = 0; l < 8; l++) {
        const double v = x(8 * k + l);
        z[k][l] = v * v;  // fma(v, v, 0)
      }
#pragma unroll
    for (int i = 32; i < N32; i += 32)
#pragma unroll
      for (int k = 0; k < 4; k++)
#pragma unroll
        for (int l = 0; l < 8; l++) {
          const double v = x(i + 8 * k + l);
          z[k][l] = __builtin_fma(v, v, z[k][l]);
        }
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int l = 0; l < 4; l++) acc[k][l] = z[k][l] + z[k][l + 4];
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int l = 0; l < 4; l++) acc[k][l] = 0.;
  }
#pragma unroll
  for (int i = N32; i < N1; i += 16)
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int l = 0; l < 4; l++) {
        const double v = x(i + 4 * k + l);
        acc[k][l] = __builtin_fma(v, v, acc[k][l]);
      }
  double dot = 0.;
  if constexpr (N1 > 0) {
    double sl[4];
#pragma unroll
    for (int l = 0; l < 4; l++) sl[l] = ((acc[0][l] + acc[1][l]) + acc[2][l]) + acc[3][l];
    dot = (sl[0] + sl[2]) + (sl[1] + sl[3]);
  }
#pragma unroll
  for (int f = N1; f < N; f++) {
    const double v = x(f);
    dot = __builtin_fma(v, v, dot);
  }
  return dot;
}

template <int N, class T>
__device__ __forceinline__ double pw_sum(T &&term) {
  if constexpr (N <= 128) {
    return pw_block<N>(term, 0);
  } else {
    constexpr int N2 = N / 2 - (N / 2) % 8;
    static_assert(N - N2 <= 128, "single split");
    return pw_block<N2>(term, 0) + pw_block<N - N2>(term, N2);
  }
}
// runtime-length version (dense index path, n <= 167)
template <class T>
__device__ double pw_block_rt(T &&term, int off, int n) {
  if (n < 8) {
    double res = 0.;
    for (int i = 0; i < n; i++) res += term(off + i);
    return res;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; j++) r[j] = term(off + j);
  int nb = n - (n % 8), i = 8;
  for (; i < nb; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] += term(off + i + j);
  }
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; i++) res += term(off + i);
  return res;
}
template <class T>
__device__ double pw_sum_rt(T &&term, int n) {
  if (n <= 128) return pw_block_rt(term, 0, n);
  int n2 = n / 2;
  n2 -= n2 % 8;
  return pw_block_rt(term, 0, n2) + pw_block_rt(term, n2, n - n2);
}

// ------------------------------------------------------------------------------------------
// wave helpers (64 lanes)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_min_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// lexicographic (d, idx) minimum across the wave; every lane gets the result
__device__ __forceinline__ void wave_min_di(double &d, int64_t &idx) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    double od = __shfl_xor(d, o, 64);
    int64_t oi = __shfl_xor(idx, o, 64);
    if (od < d || (od == d && oi < idx)) {
      d = od;
      idx = oi;
    }
  }
}

// ------------------------------------------------------------------------------------------
// K0: per-(part, channel) means of the A-side images (deterministic tree reduction)
// ------------------------------------------------------------------------------------------
// grid (IA_MEAN_CHUNKS, 4 CH): workgroup (b, part*CH + ch) sums chunk b of that image's pixels
// (fixed-order strided loop + tree), then k_part_means_fold adds the chunks in order: the same
// value on every run (a deterministic centring; any fixed mu keeps the results exact)
#define IA_MEAN_CHUNKS 128
template <int CH>
__global__ void __launch_bounds__(IA_WG) k_part_means(Imgs A, int n_ap, double *part_sums) {
  const int pc = blockIdx.y, part = pc / CH, ch = pc % CH, b = blockIdx.x;
  const double *base = part == 0 ? A.p0 : part == 1 ? A.p1 : part == 2 ? A.p2 : A.p3;
  int64_t npx = (part & 1) ? (int64_t)A.h * A.w : (int64_t)A.hc * A.wc;
  if (part >= 2) npx *= n_ap;  // A' images are contiguous
  const int64_t i0 = npx * b / IA_MEAN_CHUNKS, i1 = npx * (b + 1) / IA_MEAN_CHUNKS;
  double s = 0.;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += IA_WG) s += base[i * CH + ch];
  __shared__ double red[IA_WG];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = IA_WG / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part_sums[pc * IA_MEAN_CHUNKS + b] = red[0];
}
template <int CH>
__global__ void __launch_bounds__(IA_WG) k_part_means_fold(Imgs A, int n_ap, const double *part_sums, double *mu_part) {
  const int pc = threadIdx.x;
  if (pc >= 4 * CH) return;
  const int part = pc / CH;
  int64_t npx = (part & 1) ? (int64_t)A.h * A.w : (int64_t)A.hc * A.wc;
  if (part >= 2) npx *= n_ap;
  double s = 0.;
  for (int b = 0; b < IA_MEAN_CHUNKS; b++) s += part_sums[pc * IA_MEAN_CHUNKS + b];
  mu_part[pc] = s / (double)npx;
}

// ------------------------------------------------------------------------------------------
// K1: DB tiles of this rank's shard (one thread per DB row)
// ------------------------------------------------------------------------------------------
template <int CH>
__global__ void __launch_bounds__(IA_WG) k_db_build(LevelGeo g, Imgs A, const double *__restrict__ mu_part,
                                                     float4 *__restrict__ db, unsigned *__restrict__ Rbits) {
  using G = Geo<CH>;
  const int64_t pos = (int64_t)g.tile0 * IA_TILE + (int64_t)blockIdx.x * IA_WG + threadIdx.x;
  if (pos >= (int64_t)g.tile1 * IA_TILE) return;
  const int64_t ltile = pos / IA_TILE - g.tile0;
  const int j = (int)(pos % IA_TILE);
  const int64_t row = ia_pos_row_t(pos, g.n_tiles, g.pos2row);
  const bool real = row < g.NA;
  int img = 0, pr = 0, pc = 0;
  if (real) {
    const unsigned hw = (unsigned)g.ah * (unsigned)g.aw;
    img = (int)((unsigned)row / hw);
    const unsigned rem = (unsigned)row - (unsigned)img * hw;
    pr = (int)(rem / (unsigned)g.aw);
    pc = (int)(rem - (unsigned)pr * (unsigned)g.aw);
  }
  const Px P = make_px<CH>(A, pr, pc);
  double norm = 0.;
#pragma unroll
  for (int h = 0; h < 2; h++) {
#pragma unroll
    for (int p = 0; p < G::KP; p++) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int f = h * G::KH + 4 * p + e;
        if (f < G::D) {
          double a = 0.;
          if (real) {
            a = featp<CH>(A, P, f, img) - mu_part[feat_part<CH>(f) * CH + feat_ch<CH>(f)];
            norm += a * a;
          }
          v[e] = (float)a;
        } else if (f == G::D) {
          v[e] = real ? (float)norm : IA_PAD_NORM;
        } else {
          v[e] = 0.f;
        }
      }
      db[(ltile * G::KP + p) * IA_WAVE + h * IA_TILE + j] = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
  if (real) {
    // upper bound on |a'| (R of the certification bound), atomicMax on non-negative float bits
    float R = (float)(sqrt(norm) * (1.0 + 1e-6)) ;
    atomicMax(Rbits, __float_as_uint(R));
  }
}

// ------------------------------------------------------------------------------------------
// K1b: the fp64 feature DB, row-major (row = img*h*w + r*w + c, stride Geo::DS doubles, the
// tail zero), holding the exact pixel values of create_index's As rows (algorithms.py:63-67).
// The merge reranks candidates from it with contiguous 16-byte loads instead of re-gathering
// four symmetric-padded images per row.
// ------------------------------------------------------------------------------------------
// One wave per 64 consecutive DB rows (= raster pixels of one A' image, so lane-adjacent rows are
// pixel-adjacent): every feature load of the wave reads 64 consecutive image values (coalesced),
// the rows are assembled in LDS (odd row stride: conflict-light) and leave as one contiguous
// 64 * DS * 8 B block of 1 KiB global_store_dwordx4 per instruction.
template <int CH>
__global__ void __launch_bounds__(IA_WAVE) k_db64_build(LevelGeo g, Imgs A, double *__restrict__ db64) {
  using G = Geo<CH>;
  constexpr int DS = G::DS, LS = DS + 1, H2 = DS / 2;
  __shared__ double t[IA_WAVE * LS];
  const int64_t r0 = (int64_t)blockIdx.x * IA_WAVE;
  const int lane = threadIdx.x;
  const int64_t row = r0 + lane;
  if (row < g.NA) {
    const unsigned hw = (unsigned)g.ah * (unsigned)g.aw;
    const int img = (int)((unsigned)row / hw);
    const unsigned rem = (unsigned)row - (unsigned)img * hw;
    const int pr = (int)(rem / (unsigned)g.aw), pc = (int)(rem - (unsigned)pr * (unsigned)g.aw);
    const Px P = make_px<CH>(A, pr, pc);
    double v[G::D];
#pragma unroll
    for (int f = 0; f < G::D; f++) v[f] = featp<CH>(A, P, f, img);  // all loads in flight together
#pragma unroll
    for (int f = 0; f < DS; f++) t[lane * LS + f] = f < G::D ? v[f] : 0.;
  }
  __syncthreads();
  const int nrows = (int)min<int64_t>(IA_WAVE, g.NA - r0);
  double2 *dst = reinterpret_cast<double2 *>(db64 + r0 * DS);
  for (int i = lane; i < nrows * H2; i += IA_WAVE) {
    const int rr = i / H2, cc = 2 * (i - rr * H2);
    dst[i] = make_double2(t[rr * LS + cc], t[rr * LS + cc + 1]);
  }
}

// ------------------------------------------------------------------------------------------
// K2: queries of one wavefront step (one wave per query pixel)
// ------------------------------------------------------------------------------------------
template <int CH>
__device__ __forceinline__ void put_qfrag(float *qf, int m, int f, float v) {
  using G = Geo<CH>;
  const int qt = m / IA_TILE, j = m % IA_TILE, h = f / G::KH, s = f % G::KH;
  qf[(((int64_t)qt * G::KP + s / 4) * IA_WAVE + h * IA_TILE + j) * 4 + (s % 4)] = v;
}

template <int CH, class JS>
__global__ void __launch_bounds__(IA_WG) k_gather_query(LevelGeo g, StepDesc sd, Imgs B, JS jobs,
                                                         const double *__restrict__ mu_part,
                                                         double *__restrict__ q64, double *__restrict__ qn2,
                                                         float *__restrict__ qf) {
  using G = Geo<CH>;
  const int lane = threadIdx.x & 63;
  const int m = __builtin_amdgcn_readfirstlane(blockIdx.x * (IA_WG / IA_WAVE) + (threadIdx.x >> 6));  // wave-uniform
  if (m >= sd.Mpad) return;
  if (m >= sd.J * sd.M) {
    for (int f = lane; f < G::DP; f += IA_WAVE) put_qfrag<CH>(qf, m, f, 0.f);
    return;
  }
  const QPix px = ia_qpix(sd, g.bw, m);
  if constexpr (!JS::single) B = job_imgs(B, jobs.get(px.job));  // single job: B already holds its images
  const int r = px.r, c = px.c;
  double ss = 0.;
  for (int f = lane; f < G::DP; f += IA_WAVE) {
    if (f < G::D) {
      const double v = feat<CH>(B, f, r, c, 0);
      q64[(int64_t)m * G::D + f] = v;
      const double qc = v - mu_part[feat_part<CH>(f) * CH + feat_ch<CH>(f)];
      ss += qc * qc;
      put_qfrag<CH>(qf, m, f, -2.f * (float)qc);
    } else {
      put_qfrag<CH>(qf, m, f, f == G::D ? 1.f : 0.f);
    }
  }
  ss = wave_sum_d(ss);
  if (lane == 0) qn2[m] = ss;
}

// ------------------------------------------------------------------------------------------
// K3: MFMA distance scan with fused top-2 / threshold (the hot kernel)
//
// grid.x = nwg workgroups of 4 waves; WG w owns DB tiles [w*tpw, (w+1)*tpw) of the shard,
// wave v takes tiles w*tpw + v, +4, ... .  QT query tiles (32 queries each) are staged in
// LDS once; each DB tile is loaded once into registers (KH floats per lane) and contracted
// against every query tile:  C[row][query] = sum_k DB[row][k] * Qf[k][query]
//   A operand = DB row (lane & 31), B operand = query (lane & 31), k-half = lane >> 5;
//   C layout: lane holds query (lane & 31), rows (r&3) + 8(r>>2) + 4(lane>>5), r = 0..15.
// Each lane keeps, per query tile, the best (value, row) and the second-smallest value of
// the rows it has seen ("subset" = lane half x wave); the workgroup merges its 8 subsets into
// a top-2 list + threshold T (every unlisted row of the chunk has approx value >= T).
// ------------------------------------------------------------------------------------------
#include "ia_top2.h"

template <int KH, int QT>
__global__ void __launch_bounds__(IA_WG, 2)
k3_dist(const float4 *__restrict__ db, const float4 *__restrict__ qf, int n_tiles, int tpw, int qt0, int M,
        int nwg, int row0, int NT, float4 *__restrict__ rec, float *__restrict__ recT) {
  constexpr int KP = KH / 4;
  extern __shared__ float4 lds[];  // QT * KP * 64 float4 (queries), reused for the merge
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5;
  const int wg = blockIdx.x;

  const float4 *qsrc = qf + (int64_t)qt0 * KP * IA_WAVE;
  for (int i = threadIdx.x; i < QT * KP * IA_WAVE; i += IA_WG) lds[i] = qsrc[i];
  __syncthreads();

  float b1[QT], b2[QT];
  int i1[QT];
#pragma unroll
  for (int q = 0; q < QT; q++) {
    b1[q] = FLT_MAX;
    b2[q] = FLT_MAX;
    i1[q] = 0x7fffffff;
  }

  const int t_begin = wg * tpw, t_end = min(n_tiles, t_begin + tpw);
  int t = t_begin + wave;
  float a[KH], an[KH];
  {
    const int tl = min(t, n_tiles - 1);
    const float4 *src = db + (int64_t)tl * KP * IA_WAVE + lane;
#pragma unroll
    for (int p = 0; p < KP; p++) {
      float4 v = src[p * IA_WAVE];
      a[4 * p] = v.x; a[4 * p + 1] = v.y; a[4 * p + 2] = v.z; a[4 * p + 3] = v.w;
    }
  }
  for (; t < t_end; t += 4) {
    {  // prefetch the next tile of this wave (clamped: always issue, never branch per load)
      const int tl = min(t + 4, n_tiles - 1);
      const float4 *src = db + (int64_t)tl * KP * IA_WAVE + lane;
#pragma unroll
      for (int p = 0; p < KP; p++) {
        float4 v = src[p * IA_WAVE];
        an[4 * p] = v.x; an[4 * p + 1] = v.y; an[4 * p + 2] = v.z; an[4 * p + 3] = v.w;
      }
    }
    const int rbase = row0 + t * IA_TILE + 4 * half;
    asm volatile("" ::: "memory");  // LDS query fragments are re-read per tile, not hoisted
    // Query tiles go in pairs (two independent accumulation chains share each DB operand);
    // the top-2 epilogue of pair j is issued after the MFMAs of pair j+1 so the scheduler can
    // fill the MFMA gaps with it (distinct accumulators, no dependency).
    // Epilogue per value v (4 VALU): c = v < b1;  b2 = med3(b1, b2, v) (b1 <= b2 => the
    // second smallest of the three);  b1 = c ? v : b1;  i1 = c ? row : i1.
    f32x16 e0, e1;
    auto epilogue = [&](const f32x16 &acc, int q) {
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const float v = acc[r];
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        const bool c = v < b1[q];
        b2[q] = __builtin_amdgcn_fmed3f(b1[q], b2[q], v);
        b1[q] = c ? v : b1[q];
        i1[q] = c ? row : i1[q];
      }
    };
#pragma unroll
    for (int qp = 0; qp < QT; qp += 2) {
      constexpr f32x16 zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const bool two = qp + 1 < QT;
      f32x16 c0 = zero, c1 = zero;
      const float4 *qb0 = lds + qp * KP * IA_WAVE + lane;
      const float4 *qb1 = qb0 + KP * IA_WAVE;
#pragma unroll
      for (int p = 0; p < KP; p++) {
        const float4 x0 = qb0[p * IA_WAVE];
        const float4 x1 = two ? qb1[p * IA_WAVE] : x0;
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * p], x0.x, c0, 0, 0, 0);
        if (two) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * p], x1.x, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * p + 1], x0.y, c0, 0, 0, 0);
        if (two) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * p + 1], x1.y, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * p + 2], x0.z, c0, 0, 0, 0);
        if (two) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * p + 2], x1.z, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * p + 3], x0.w, c0, 0, 0, 0);
        if (two) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * p + 3], x1.w, c1, 0, 0, 0);
      }
      if (qp >= 2) {
        epilogue(e0, qp - 2);
        epilogue(e1, qp - 1);
      }
      e0 = c0;
      e1 = c1;
    }
    {
      constexpr int ql = ((QT - 1) / 2) * 2;  // first tile of the last pair
      epilogue(e0, ql);
      if (ql + 1 < QT) epilogue(e1, ql + 1);
    }
#pragma unroll
    for (int k = 0; k < KH; k++) a[k] = an[k];
  }

  // ---- merge the 8 subsets of each query: lane halves by shuffle, waves through LDS
  __syncthreads();  // queries no longer needed: reuse LDS
  Top2 *red = reinterpret_cast<Top2 *>(lds);  // [4 waves][QT][32]
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
  for (int x = threadIdx.x; x < QT * IA_TILE; x += IA_WG) {
    Top2 m = red[x];
#pragma unroll
    for (int w = 1; w < 4; w++) m = top2_merge(m, red[(w * QT) * IA_TILE + x]);
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
// Split-f16 matcher (IA_MATCH_F16X3): K1h / K2h / K3h
//
// Every operand x (centred DB feature a', |a'|^2/256, query -2q', 256) is split into
// hi = f16(f32(x)) and lo = f16(f32(x) - hi) (22 significant bits together); K3h sums
// lo_a*hi_q + hi_a*lo_q + hi_a*hi_q with v_mfma_f32_32x32x16_f16 (f16 products are exact in
// fp32), i.e. 3 f16 MFMAs replace 8 f32 ones per 16 k.  The value carries a larger, still
// rigorous, error bound (ia_eps_c_h), so K4's certification keeps the NN exact.
// Fragment order (tile of 32 DB rows or 32 queries, k-step s of 16, part 0 = hi / 1 = lo):
//   h16x8 piece p = 2s + part, lane L:  row (L & 31), k = 16s + 8(L >> 5) + e, e = 0..7
// ------------------------------------------------------------------------------------------

__device__ __forceinline__ void split_h(double x, _Float16 &hi, _Float16 &lo) {
  const float xf = (float)x;
  const _Float16 h = (_Float16)xf;
  hi = h;
  lo = (_Float16)(xf - (float)h);  // exact in fp32: xf and h share the leading bits
}

// max |x| over the level's images (decides whether every operand fits f16, IA_F16_MAXABS)
struct AbsArrays {
  const double *p[8];
  int64_t n[8];
};
__global__ void __launch_bounds__(IA_WG) k_absmax(AbsArrays arr, unsigned *__restrict__ out) {
  float m = 0.f;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const double *p = arr.p[k];
    const int64_t n = arr.n[k];
    for (int64_t i = (int64_t)blockIdx.x * IA_WG + threadIdx.x; i < n; i += (int64_t)gridDim.x * IA_WG)
      m = fmaxf(m, (float)fabs(p[i]));  // NaN propagates as "not finite" below
  }
  if (!(m <= 3.0e38f)) m = 3.4e38f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));
}

// One wave per DB tile (32 rows x 64 columns in v_mfma_f32_32x32x16_f16 operand order): lane L
// (row j = L & 31, column half h = L >> 5) holds columns 16s + 8h .. + 7 of every k-step s, i.e.
// 64 contiguous bytes of its row in the fp64 row DB (K1b, written just before: rows are whole
// 128 B lines, no image gathers).  Centre by mu, |a'|^2 = the two lane halves' partial sums (the
// certified bound does not depend on its rounding order), split into f16 hi + lo, and store
// each piece as one 1 KiB coalesced wave store.  Grid-stride over tiles: one atomicMax of R per
// workgroup.
template <int CH, int KS>
__global__ void __launch_bounds__(IA_WG) k_db_build_h(LevelGeo g, const double *__restrict__ db64,
                                                       const double *__restrict__ mu_part, h16x8 *__restrict__ db,
                                                       unsigned *__restrict__ Rbits) {
  constexpr int D = 55 * CH, DS = Geo<CH>::DS;
  static_assert(16 * KS >= D + 1, "k-steps must hold D features + the norm column");
  static_assert(DS % 8 == 0, "64-byte row pieces");
  __shared__ float wR[IA_WG / IA_WAVE];
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  const int64_t nloc = (int64_t)g.tile1 - g.tile0;
  double mu[KS][8];  // this lane's feature means (the lane's columns are fixed)
#pragma unroll
  for (int s = 0; s < KS; s++)
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const int f = 16 * s + 8 * h + e;
      mu[s][e] = f < D ? mu_part[feat_part<CH>(f) * CH + feat_ch<CH>(f)] : 0.;
    }
  float Rmax = 0.f;
  for (int64_t lt = (int64_t)blockIdx.x * (IA_WG / IA_WAVE) + wave; lt < nloc; lt += (int64_t)gridDim.x * (IA_WG / IA_WAVE)) {
    const int64_t pos = (g.tile0 + lt) * IA_TILE + j;
    const int64_t row = ia_pos_row_t(pos, g.n_tiles, g.pos2row);
    const bool real = row < g.NA;
    double a[KS][8];
#pragma unroll
    for (int s = 0; s < KS; s++) {
      const int f0 = 16 * s + 8 * h;
      double2 v[4];
      if (real && f0 < DS) {
        const double2 *src = reinterpret_cast<const double2 *>(db64 + row * DS + f0);
#pragma unroll
        for (int e = 0; e < 4; e++) v[e] = src[e];
      } else {
#pragma unroll
        for (int e = 0; e < 4; e++) v[e] = make_double2(0., 0.);
      }
#pragma unroll
      for (int e = 0; e < 4; e++) {
        a[s][2 * e] = v[e].x;
        a[s][2 * e + 1] = v[e].y;
      }
    }
    double nrm = 0.;
#pragma unroll
    for (int s = 0; s < KS; s++)
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const int f = 16 * s + 8 * h + e;
        a[s][e] = f < D ? a[s][e] - mu[s][e] : 0.;
        nrm += a[s][e] * a[s][e];
      }
    nrm += __shfl_xor(nrm, 32, 64);  // both halves: p0 + p1 (addition commutes exactly)
    const int64_t tb = lt * TileFmt<KS>::STRIDE;
#pragma unroll
    for (int s = 0; s < KS; s++) {
      h16x8 vh, vl;
#pragma unroll
      for (int e = 0; e < 8; e++) {
        double x = a[s][e];
        if (16 * s + 8 * h + e == D) x = real ? nrm * (1.0 / IA_NORM_SCALE) : 60000.0;  // padding rows: never a candidate
        _Float16 hi, lo;
        split_h(x, hi, lo);
        vh[e] = hi;
        vl[e] = lo;
      }
      if (!(TileFmt<KS>::CMP && s == KS - 1 && h == 1)) {  // (compact: padding half not stored)
        db[tb + TileFmt<KS>::off(2 * s, lane)] = vh;
        db[tb + TileFmt<KS>::off(2 * s + 1, lane)] = vl;
      }
    }
    if (real) Rmax = fmaxf(Rmax, (float)(sqrt(nrm) * (1.0 + 1e-6)));
  }
  // R = max |a'| (certification bound): wave, then workgroup max, one atomic per workgroup
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) Rmax = fmaxf(Rmax, __shfl_xor(Rmax, o, 64));
  if (lane == 0) wR[wave] = Rmax;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = wR[0];
#pragma unroll
    for (int w = 1; w < IA_WG / IA_WAVE; w++) m = fmaxf(m, wR[w]);
    if (m > 0.f) atomicMax(Rbits, __float_as_uint(m));
  }
}

template <int KS>
__device__ __forceinline__ void put_qh(_Float16 *qf, int m, int f, double v) {
  const int qt = m / IA_TILE, j = m % IA_TILE, s = f >> 4, h = (f >> 3) & 1, e = f & 7;
  _Float16 hi, lo;
  split_h(v, hi, lo);
  const int64_t base = (((int64_t)qt * 2 * KS + 2 * s) * IA_WAVE + h * IA_TILE + j) * 8 + e;
  qf[base] = hi;
  qf[base + IA_WAVE * 8] = lo;
}

template <int CH, int KS, class JS>
__global__ void __launch_bounds__(IA_PQ_WG) k_gather_query_h(LevelGeo g, StepDesc sd, Imgs B, JS jobs,
                                                           const double *__restrict__ mu_part,
                                                           double *__restrict__ q64, double *__restrict__ qn2,
                                                           _Float16 *__restrict__ qf) {
  constexpr int D = 55 * CH, KD = 16 * KS;
  const int lane = threadIdx.x & 63;
  const int m = __builtin_amdgcn_readfirstlane(blockIdx.x * IA_PQ_WPB + (threadIdx.x >> 6));  // wave-uniform
  if (m >= sd.Mpad) return;
  if (m >= sd.J * sd.M) {
    for (int f = lane; f < KD; f += IA_WAVE) put_qh<KS>(qf, m, f, 0.);
    return;
  }
  const QPix px = ia_qpix(sd, g.bw, m);
  if constexpr (!JS::single) B = job_imgs(B, jobs.get(px.job));  // single job: B already holds its images
  const int r = px.r, c = px.c;
  double ss = 0.;
  for (int f = lane; f < KD; f += IA_WAVE) {
    if (f < D) {
      const double v = feat<CH>(B, f, r, c, 0);
      q64[(int64_t)m * D + f] = v;
      const double qc = v - mu_part[feat_part<CH>(f) * CH + feat_ch<CH>(f)];
      ss += qc * qc;
      put_qh<KS>(qf, m, f, -2.0 * qc);
    } else {
      put_qh<KS>(qf, m, f, f == D ? IA_NORM_SCALE : 0.);
    }
  }
  ss = wave_sum_d(ss);
  if (lane == 0) qn2[m] = ss;
}

// ------------------------------------------------------------------------------------------
// K4: exact rerank + certification (+ coherence, kappa rule, writeback) — one wave / query
// ------------------------------------------------------------------------------------------
// The 55 exact features of DB row `row` (1 channel) read straight from the A-side pyramid images
// (option "row_source" = 1) instead of the fp64 row DB: row = img*h*w + r*w + c holds
// [A coarse 3x3 | A fine 5x5 | A'_img coarse 3x3 | A'_img fine, first 12] (algorithms.py:36-41,
// 63-67), the windows symmetric-padded (ia_reflect).  20 MB of images at 1024^2 instead of a
// 470 MB row DB: the rows stay cache resident and the memory-side cache is left to the MFMA DB.
__device__ __forceinline__ void row_from_imgs(const Imgs &A, int64_t row, double (&t)[56]) {
  const unsigned hw = (unsigned)A.h * (unsigned)A.w;
  const int img = (int)((unsigned)row / hw);
  const unsigned rem = (unsigned)row - (unsigned)img * hw;
  const int r = (int)(rem / (unsigned)A.w), c = (int)(rem - (unsigned)r * (unsigned)A.w);
  const Px P = make_px<1>(A, r, c);
#pragma unroll
  for (int f = 0; f < 55; f++) t[f] = featp<1>(A, P, f, img);
  t[55] = 0.;
}
// exact DB-row distance of row `row` (level path): ((a - q)**2).sum() in numpy order, the row
// read from the fp64 DB (K1b) or, with Ai (1 channel), from the images
template <int CH>
__device__ __forceinline__ double exact_dist_level(const double *__restrict__ db64, int64_t row, const double *q,
                                                   const Imgs *Ai = nullptr) {
  if constexpr (CH == 1) {
    if (Ai) {
      double t[56];
      row_from_imgs(*Ai, row, t);
      return pw_sum<55>([&](int f) {
        const double d = t[f] - q[f];
        return d * d;
      });
    }
  }
  const double *a = db64 + row * Geo<CH>::DS;
  return pw_sum<Geo<CH>::D>([&](int f) {
    const double d = a[f] - q[f];
    return d * d;
  });
}

// MFMA error bound of a row with |a'| <= Rx (ia_internal.h ia_eps_c_h / DESIGN.md §5)
__device__ __forceinline__ double merge_eps(const MergeArgs &a, double Rx, double qn) {
  return a.eps_c * (Rx * Rx + 2.0 * Rx * qn) + a.eps_a * (Rx * Rx + 14.0 * Rx + 28.0 * qn + 260.0);
}
// Certification threshold of the best exact distance bd: a chunk whose unlisted rows all have
// MFMA value >= T can hide a row that beats or ties bd only if T <= theta.  Only rows with exact
// distance <= bd matter, and such a row has |a'| <= |q'| + sqrt(bd) (|a' - q'|^2 = its distance;
// 1e-12 covers the fp64 roundings of qn and bd), so its error bound uses that radius instead of
// the DB-wide R when smaller (at 1024^2 about ten times tighter at the median query: far fewer
// near-duplicate chunks rescanned, the same certified decisions).
__device__ __forceinline__ double cert_theta(const MergeArgs &a, double R, double qn, double qn2, double bd) {
  const double Rl = fmin(R, (qn + sqrt(bd)) * (1.0 + 1e-12) + 1e-12);
  return bd - qn2 + merge_eps(a, Rl, qn) + 1e-13 * (bd + 1.0);
}

// the certified single-rank winner of query m (exact NN over this rank's shard); RPL records per
// lane (nwg <= 64 RPL)
template <int RPL = IA_WG_TARGET / IA_WAVE, class DistFn>
__device__ Winner certified_winner(const MergeArgs &a, int m, DistFn &&dist, unsigned *stat_out) {
  const int lane = threadIdx.x & 63;
  const float4 *rr = a.rec + (int64_t)m * a.nwg;
  const float *rT = a.recT + (int64_t)m * a.nwg;
  // issue every record load at once (clamped index, no per-load branch), mask afterwards
  float v1[RPL], v2[RPL], tt[RPL];
#pragma unroll
  for (int j = 0; j < RPL; j++) {
    const int w = min(lane + IA_WAVE * j, a.nwg - 1);
    const float4 x = rr[w];
    const float t = rT[w];
    const bool ok = lane + IA_WAVE * j < a.nwg;
    v1[j] = ok ? x.x : FLT_MAX;
    v2[j] = ok ? x.z : FLT_MAX;
    tt[j] = ok ? t : FLT_MAX;
  }
  const double R = (double)__uint_as_float(*a.Rbits);
  const double qn2 = a.qn2[m];
  float a1 = FLT_MAX;
#pragma unroll
  for (int j = 0; j < RPL; j++) a1 = fminf(a1, v1[j]);
  a1 = wave_min_f(a1);
  const double qn = sqrt(qn2);
  const double eps = merge_eps(a, R, qn);
  const double thr = (double)a1 + 2.0 * eps;

  // rerank every listed candidate that could be the exact winner
  unsigned cmask = 0;
#pragma unroll
  for (int j = 0; j < RPL; j++) {
    if ((double)v1[j] <= thr) cmask |= 1u << (2 * j);
    if ((double)v2[j] <= thr) cmask |= 1u << (2 * j + 1);
  }
  double bd = DBL_MAX;
  int64_t bi = INT64_MAX;
  unsigned long long nre = 0;
  while (cmask) {
    const int b = __ffs(cmask) - 1;
    cmask &= cmask - 1;
    const float4 x = rr[min(lane + IA_WAVE * (b >> 1), a.nwg - 1)];  // L2-hot re-read of the record
    const int64_t i = __float_as_int((b & 1) ? x.w : x.y);
    if (i >= 0 && i < a.NA) {
      const double d = dist(i);
      nre++;
      if (d < bd || (d == bd && i < bi)) { bd = d; bi = i; }
    }
  }
  wave_min_di(bd, bi);
  if (a.rr && bd == DBL_MAX) {
    // a shard of the pruned scan that contracted no pair for this query: none of its tiles
    // passed the bound U' (K3p computes every pair a query needs), so none of its rows can be
    // the exact NN or tie it.  No winner from this shard.
    *stat_out = 0u;
    return Winner{DBL_MAX, INT64_MAX};
  }

  // certification: every unlisted row of chunk w has MFMA value >= T_w, hence true distance
  // >= T_w + |q'|^2 - eps.  Chunks with T_w <= theta may hide a row that beats or ties bd.
  const double theta = cert_theta(a, R, qn, qn2, bd);
  const float thetaf = round_down_f(theta);  // (t <= theta  <=>  t <= theta rounded down, t a float)
  unsigned long long nfb = 0;
#pragma unroll
  for (int jb = 0; jb < RPL; jb++) {
    const int base = jb * IA_WAVE;
    unsigned long long mask = __ballot(tt[jb] <= thetaf);
    while (mask) {
      const int j = __ffsll((long long)mask) - 1;
      mask &= mask - 1;
      const int wgid = base + j;
      double cd = DBL_MAX;
      int64_t ci = INT64_MAX;
      if (a.rr) {
        // pruned scan (a shard of it): chunk = tiles wgid, wgid + nwg, ...  Rows that can
        // displace or tie the winner have exact distance <= bd, and the global NN is <= U (the
        // query's coherence candidate), so only tiles whose projection bound passes
        // min(bd * ufac, U') are rescanned.  A shard none of whose tiles passed U' in K3p holds
        // no such row: nothing is rescanned and it reports no winner (d = DBL_MAX).
        const float4 ql = a.qinfo[3 * m], qh = a.qinfo[3 * m + 1];
        const float ub = fminf(round_up_f(bd * a.ufac), a.qinfo[3 * m + 2].x);
        for (int64_t tb = 0; wgid + (int64_t)a.nwg * tb < a.NT; tb += IA_WAVE) {
          const int64_t t = wgid + (int64_t)a.nwg * (tb + lane);
          const bool nd = t < a.NT && prune_lb(a.boxes[2 * t], a.boxes[2 * t + 1], ql, qh) <= ub;
          unsigned long long nm = __ballot(nd);
          while (nm) {
            const int jt = __ffsll((long long)nm) - 1;
            nm &= nm - 1;
            if (lane < IA_TILE) {
              const int64_t i = a.pos2row[(wgid + (int64_t)a.nwg * (tb + jt)) * IA_TILE + lane];
              if (i < a.NA) {
                const double d = dist(i);
                if (d < cd || (d == cd && i < ci)) { cd = d; ci = i; }
              }
            }
          }
        }
      } else {
        const int64_t p0 = (int64_t)a.pos0 + (int64_t)wgid * a.tpw * IA_TILE;
        const int64_t p1 = min((int64_t)a.pos_end, p0 + (int64_t)a.tpw * IA_TILE);
        for (int64_t p = p0 + lane; p < p1; p += IA_WAVE) {
          const int64_t i = ia_pos_row(p, a.NT);
          if (i >= a.NA) continue;
          const double d = dist(i);
          if (d < cd || (d == cd && i < ci)) { cd = d; ci = i; }
        }
      }
      wave_min_di(cd, ci);
      if (cd < bd || (cd == bd && ci < bi)) { bd = cd; bi = ci; }
      nfb++;
    }
  }
  unsigned long long tot = nre;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
  *stat_out = (unsigned)min((unsigned long long)0xffff, tot) | ((unsigned)min((unsigned long long)0x1fff, nfb) << 16);
  return Winner{bd, bi};
}

// best_coherence_match's pick for query pixel (r, c) (algorithms.py:92-130): candidates in
// product(rows, cols) order, first argmin of the unweighted norm.  Independent of the NN winner,
// so the exchange merge runs it while the peers' winners are in flight.
struct CohPick {
  int pr, pc, img;
  bool has;
};
template <int CH>
__device__ __forceinline__ CohPick coherence_pick(const LevelGeo &g, const double *__restrict__ db64, int r, int c,
                                                  const double *q, const int32_t *__restrict__ s,
                                                  const int32_t *__restrict__ im) {
  const int lane = threadIdx.x & 63;
  const unsigned hw = (unsigned)g.ah * (unsigned)g.aw;
  const int qi = r * g.bw + c;
  CohPick k{-1, -1, 0, false};
  if (qi == 0) return k;
  double dk = DBL_MAX;
  int64_t kk = INT64_MAX;
  int cpr = -1, cpc = -1, cim = 0;
  if (lane < 15) {
    const int nr = r - 2 + lane / 5, nc = c - 2 + lane % 5;
    if (nr >= 0 && nc >= 0 && nc < g.bw && nr * g.bw + nc < qi) {
      const int nb = nr * g.bw + nc;
      const int tr = s[2 * nb] + r - nr, tc = s[2 * nb + 1] + c - nc;
      if (tr >= 0 && tr < g.ah && tc >= 0 && tc < g.aw) {
        cim = im[nb];
        cpr = tr;
        cpc = tc;
        const int64_t row = (int64_t)cim * hw + (int64_t)tr * g.aw + tc;
        dk = cr_sqrt(exact_dist_level<CH>(db64, row, q));
        kk = lane;
      }
    }
  }
  wave_min_di(dk, kk);
  if (kk != INT64_MAX) {
    const int src = (int)kk;
    k.pr = __shfl(cpr, src, 64);
    k.pc = __shfl(cpc, src, 64);
    k.img = __shfl(cim, src, 64);
    k.has = true;
  }
  return k;
}
// kappa rule + writeback for query pixel (r, c) whose NN row is app_ix and coherence pick ck
// (image_analogies.py:182-220, algorithms.py:133-135)
template <int CH>
__device__ void finish_pick(const LevelGeo &g, const Imgs &A, const double *__restrict__ db64, int r, int c,
                            int64_t app_ix, const CohPick &ck, const double *q, int32_t *__restrict__ s,
                            int32_t *__restrict__ im, double *__restrict__ Bp, const double *__restrict__ weights, double kf,
                            unsigned *pstat, unsigned stat, int32_t *__restrict__ nn = nullptr) {
  constexpr int D = Geo<CH>::D;
  const int lane = threadIdx.x & 63;
  const unsigned hw = (unsigned)g.ah * (unsigned)g.aw;
  const int qi = r * g.bw + c;
  int img = (int)((unsigned)app_ix / hw);
  const unsigned rem = (unsigned)app_ix - (unsigned)img * hw;
  int pr = (int)(rem / (unsigned)g.aw), pc = (int)(rem - (unsigned)pr * (unsigned)g.aw);
  bool coh_won = false, kamb = false;
  if (ck.has) {
    // compute_distance(AAp_feat, BBp_feat, weights) = norm((a - q) * w)**2 for app and coh
    double part = 0.;
    if (lane < 2) {
      const int ii = lane == 0 ? img : ck.img, rr_ = lane == 0 ? pr : ck.pr, cc_ = lane == 0 ? pc : ck.pc;
      const double *arow = db64 + ((int64_t)ii * hw + (int64_t)rr_ * g.aw + cc_) * Geo<CH>::DS;
      part = blas_dot_sq<D>([&](int f) { return (arow[f] - q[f]) * weights[f]; });
      part = cr_sqrt(part);
    }
    const double y_app = __shfl(part, 0, 64), y_coh = __shfl(part, 1, 64);
    const double d_app = y_app * y_app, d_coh = y_coh * y_coh;
    kamb = kappa_ambiguous(y_app, d_app, y_coh, d_coh, kf);
    if (d_coh <= d_app * kf) {
      img = ck.img;
      pr = ck.pr;
      pc = ck.pc;
      coh_won = true;
    }
  }
  if (lane < CH) Bp[(int64_t)qi * CH + lane] = A.p3[img * A.img_stride_f + ((int64_t)pr * g.aw + pc) * CH + lane];
  if (lane == 0) {
    s[2 * qi] = pr;
    s[2 * qi + 1] = pc;
    im[qi] = img;
    if (pstat) pstat[qi] = stat | (kamb ? 1u << 29 : 0u) | (coh_won ? 1u << 30 : 0u);
    if (nn) nn[qi] = app_ix >= 0 && app_ix < (int64_t)g.NA ? (int)app_ix : -1;  // option "nn_bound"
  }
}
// coherence + kappa + writeback for query pixel (r, c) whose NN row is app_ix
template <int CH>
__device__ void finish_pixel(const LevelGeo &g, const Imgs &A, const double *__restrict__ db64, int r, int c, int64_t app_ix,
                             const double *q,
                             int32_t *__restrict__ s, int32_t *__restrict__ im, double *__restrict__ Bp,
                             const double *__restrict__ weights, double kf, unsigned *pstat, unsigned stat,
                             int32_t *__restrict__ nn = nullptr) {
  const CohPick ck = coherence_pick<CH>(g, db64, r, c, q, s, im);
  finish_pick<CH>(g, A, db64, r, c, app_ix, ck, q, s, im, Bp, weights, kf, pstat, stat, nn);
}

// Both distances of DB row `row` against query q from ONE set of feature loads (the row of the
// fp64 DB, K1b; q and w staged in LDS by the caller):
//   unw = ((a - q)**2).sum()  in numpy's pairwise order (NN rerank / coherence ranking)
//   wsq = sum(((a - q) * w)**2) sequentially (compute_distance before its sqrt / square)
template <int CH>
__device__ __forceinline__ void row_dists(const double *__restrict__ db64, int row, const double *q, const double *w,
                                          double &unw, double &wsq, const Imgs *Ai = nullptr) {
  constexpr int D = Geo<CH>::D, DS = Geo<CH>::DS;
  const double *a = db64 + (int64_t)row * DS;
  if constexpr (CH == 1) {
    double t[D + 1];
    if (Ai) {
      row_from_imgs(*Ai, row, t);
    } else {
      const double2 *a2 = reinterpret_cast<const double2 *>(a);
#pragma unroll
      for (int k = 0; k < (D + 1) / 2; k++) {  // all 28 loads issued before any use
        const double2 v = a2[k];
        t[2 * k] = v.x;
        t[2 * k + 1] = v.y;
      }
    }
#pragma unroll
    for (int f = 0; f < D; f++) t[f] -= q[f];
    unw = pw_sum<D>([&](int f) { return t[f] * t[f]; });
    wsq = blas_dot_sq<D>([&](int f) { return t[f] * w[f]; });
  } else {  // 165 doubles do not fit in registers: read the row twice
    unw = pw_sum<D>([&](int f) {
      const double d = a[f] - q[f];
      return d * d;
    });
    wsq = blas_dot_sq<D>([&](int f) { return (a[f] - q[f]) * w[f]; });
  }
}

// row of the lowest set candidate bit (bit 2j: record j's best, bit 2j+1: its runner-up)
template <int RPL>
__device__ __forceinline__ int lowest_cand(unsigned cmask, const int (&i1)[RPL], const int (&i2)[RPL],
                                           const float (&v1)[RPL], const float (&v2)[RPL], float &v) {
  int row = -1;
  v = FLT_MAX;
#pragma unroll
  for (int j = RPL - 1; j >= 0; j--) {
    const bool b2 = (cmask >> (2 * j + 1)) & 1, b1 = (cmask >> (2 * j)) & 1;
    row = b2 ? i2[j] : row;
    v = b2 ? v2[j] : v;
    row = b1 ? i1[j] : row;
    v = b1 ? v1[j] : v;
  }
  return row;
}

// ---- cross-lane exchange without LDS: partner of step k of a 64-lane butterfly -----------------
// steps 0-3 stay inside a 16-lane row (DPP quad_perm xor 1, xor 2, row_half_mirror,
// row_mirror), 4 pairs rows 0-1 / 2-3 (v_permlane16_swap), 5 the two wave halves
// (v_permlane32_swap).  Every lane's partner differs from it and the pairing at each step
// joins two groups that are each already reduced, so after step 5 every lane holds the
// reduction of all 64.
template <int STEP>
__device__ __forceinline__ int lane_xchg(int v) {
  if constexpr (STEP == 0) return __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false);
  else if constexpr (STEP == 1) return __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false);
  else if constexpr (STEP == 2) return __builtin_amdgcn_update_dpp(v, v, 0x141, 0xF, 0xF, false);
  else if constexpr (STEP == 3) return __builtin_amdgcn_update_dpp(v, v, 0x140, 0xF, 0xF, false);
  else if constexpr (STEP == 4) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    return (int)(((threadIdx.x >> 4) & 1) ? r[0] : r[1]);
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
    return (int)((threadIdx.x & 32) ? r[0] : r[1]);
  }
}
template <int STEP>
__device__ __forceinline__ double lane_xchg_d(double v) {
  const int lo = lane_xchg<STEP>(__double2loint(v)), hi = lane_xchg<STEP>(__double2hiint(v));
  return __hiloint2double(hi, lo);
}
template <int STEP>
__device__ __forceinline__ float lane_xchg_f(float v) {
  return __int_as_float(lane_xchg<STEP>(__float_as_int(v)));
}
// lexicographic (d, i) minimum across the wave for TWO independent keys at once
template <int STEP = 0>
__device__ __forceinline__ void wave_min2_di(double &d0, int &i0, double &d1, int &i1) {
  if constexpr (STEP < 6) {
    const double e0 = lane_xchg_d<STEP>(d0), e1 = lane_xchg_d<STEP>(d1);
    const int j0 = lane_xchg<STEP>(i0), j1 = lane_xchg<STEP>(i1);
    if (e0 < d0 || (e0 == d0 && j0 < i0)) { d0 = e0; i0 = j0; }
    if (e1 < d1 || (e1 == d1 && j1 < i1)) { d1 = e1; i1 = j1; }
    wave_min2_di<STEP + 1>(d0, i0, d1, i1);
  }
}
template <int STEP = 0>
__device__ __forceinline__ float wave_min_f_x(float v) {
  if constexpr (STEP < 6) return wave_min_f_x<STEP + 1>(fminf(v, lane_xchg_f<STEP>(v)));
  else return v;
}
// v of lane l (wave-uniform l): two v_readlane, no LDS crossbar (a __shfl is a ds_bpermute)
__device__ __forceinline__ double readlane_d(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ int lane_prefix(unsigned long long bal) {  // set bits of bal below this lane
  return __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
}
template <int STEP = 0>
__device__ __forceinline__ double wave_min_d_x(double v) {
  if constexpr (STEP < 6) return wave_min_d_x<STEP + 1>(fmin(v, lane_xchg_d<STEP>(v)));
  else return v;
}
template <int STEP = 0>
__device__ __forceinline__ double wave_sum_d_x(double v) {  // fixed butterfly order: deterministic
  if constexpr (STEP < 6) return wave_sum_d_x<STEP + 1>(v + lane_xchg_d<STEP>(v));
  else return v;
}

// The two pixels of step t whose results a fused K4(t) + K2p(t + 1) wave (k_merge_gather) hands
// to its next query: its own (r0, c0) and the row above's (r1, c1), both written in the same
// launch, so their B', s and im come from registers / the handoff slot, never from memory.
struct QHand {
  int r0 = -1, c0 = -1, r1 = -1, c1 = -1;
  double v0 = 0., v1 = 0.;
  int s0r = 0, s0c = 0, i0 = 0, s1r = 0, s1c = 0, i1 = 0;
  int n0 = -1, n1 = -1;  // their exact NN rows (option "nn_bound")
};
template <bool FUSE>
__device__ __forceinline__ double feat_q1(const Imgs &B, int f, int r, int c, const QHand &h) {
  if constexpr (FUSE) {
    if (f >= 43) {  // the B' part (causal 5x5 at (r, c), k < 12)
      const int k = f - 43, y = ia_reflect(r + k / 5 - 2, B.h), x = ia_reflect(c + k % 5 - 2, B.w);
      if (y == h.r0 && x == h.c0) return h.v0;
      if (y == h.r1 && x == h.c1) return h.v1;
      return B.p3[(int64_t)y * B.w + x];
    }
  }
  return feat<1>(B, f, r, c, 0);
}

// owner-computes sharded step (XOPub): query m's fragments (16 h16x8 pieces from LDS, one store
// instruction per area), its pruning record, then - once those stores completed - its seq, into
// every rank's area
// lane k < 3 picks record k, component by component (a float4 chosen by a lane-dependent
// ternary becomes a dynamically indexed private array: scratch, and a scratch-using kernel)
__device__ __forceinline__ float4 sel3(int k, const float4 &a, const float4 &b, const float4 &c) {
  return make_float4(k == 0 ? a.x : k == 1 ? b.x : c.x, k == 0 ? a.y : k == 1 ? b.y : c.y,
                     k == 0 ? a.z : k == 1 ? b.z : c.z, k == 0 ? a.w : k == 1 ? b.w : c.w);
}
template <int KS>
__device__ __forceinline__ void xo_publish(const XOPub &xp, int m, int lane, const _Float16 *xh0, const _Float16 *xh1,
                                           float4 i0, float4 i1, float4 i2) {
  __builtin_amdgcn_wave_barrier();  // xh written by this wave's lanes
  const int qt = m / IA_TILE, j = m % IA_TILE;
  const int c = lane, sp = c >> 2, part = (c >> 1) & 1, h = c & 1;  // chunk c < 2 KS * 2
  h16x8 v{};
  if (c < 4 * KS) v = *reinterpret_cast<const h16x8 *>(&(part ? xh1 : xh0)[16 * sp + 8 * h]);
  const int64_t t0 = xp.slot0 / IA_TILE;
  for (int o = 0; o < xp.W; o++) {
    if (c < 4 * KS)
      reinterpret_cast<h16x8 *>(xp.area[o] + XOLayout::FRAG)[((t0 + qt) * 2 * KS + 2 * sp + part) * IA_WAVE + h * IA_TILE + j] = v;
    if (lane < 3) reinterpret_cast<float4 *>(xp.area[o] + XOLayout::INFO)[3 * (xp.slot0 + m) + lane] = sel3(lane, i0, i1, i2);
  }
  ia_stores_done();
  if (lane < xp.W)
    __hip_atomic_store(reinterpret_cast<unsigned *>(xp.area[lane] + XOLayout::QSEQ) + xp.slot0 + m, xp.seq, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// option "fuse_sort" (NextStep::kslot): query m of step nx.sn publishes its sort key (the Morton
// key's top 20 bits above the 12-bit query index, k_query_sort's order), waits for every key of
// the step, takes its rank x among them and writes its pruning record, query index and split-f16
// fragments (hi / lo columns from xh0 / xh1) at sorted slot x.  Every query of the step is
// gathered by exactly one wave of this launch, all of them resident together (one wave per
// workgroup), so the wait drains; a key that never arrives (bounded, 20 s) sets err bit 4.
template <int KS>
__device__ __forceinline__ void sorted_publish(const NextStep &nx, int m, int lane, const _Float16 *xh0, const _Float16 *xh1,
                                               float4 i0, float4 i1, float4 i2) {
  const unsigned key = (__float_as_uint(i2.y) & 0xFFFFF000u) | (unsigned)m;
  if (lane == 0)
    __hip_atomic_store(nx.kslot + m, ((unsigned long long)nx.seq << 32) | key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_wave_barrier();  // xh written by this wave's lanes
  // the fragments to registers while the other keys arrive
  const int c = lane, sp = c >> 2, part = (c >> 1) & 1, h = c & 1;  // chunk c < 4 KS
  h16x8 v{};
  if (c < 4 * KS) v = *reinterpret_cast<const h16x8 *>(&(part ? xh1 : xh0)[16 * sp + 8 * h]);
  int below = 0;
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  const bool late = __hip_atomic_load(nx.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
  for (int i = lane; i < nx.sn.Mpad; i += IA_WAVE) {
    unsigned long long x;
    // relaxed: the slots are uncached (no stale line to invalidate)
    while (((x = __hip_atomic_load(nx.kslot + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) >> 32) != nx.seq && !late) {
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > nx.timeout_ticks) {
        atomicOr(nx.err, 16u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    below += (unsigned)x < key ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) below += __shfl_xor(below, o, 64);
  const int x = __builtin_amdgcn_readfirstlane(below);
  const int qt = x / IA_TILE, j = x % IA_TILE;
  if (c < 4 * KS) reinterpret_cast<h16x8 *>(nx.sfrag)[((int64_t)qt * 2 * KS + 2 * sp + part) * IA_WAVE + h * IA_TILE + j] = v;
  if (lane < 3) nx.sinfo[3 * x + lane] = sel3(lane, i0, i1, i2);
  if (lane == 3) nx.sorder[x] = m;
}

// K2p's pad query m >= J M: zero fragments, an empty pruning record
template <int KS>
__device__ __forceinline__ void gather_p_pad(int m, int lane, _Float16 *qf, float4 *qinfo, float4 &o0, float4 &o1,
                                             float4 &o2) {
  if (lane < 16 * KS) put_qh<KS>(qf, m, lane, 0.);
  o0 = o1 = make_float4(0.f, 0.f, 0.f, 0.f);
  o2 = make_float4(-INFINITY, __uint_as_float(IA_PRUNE_KEY_PAD), -INFINITY, 0.f);
  if (lane == 0) {
    qinfo[3 * m] = o0;
    qinfo[3 * m + 1] = o1;
    qinfo[3 * m + 2] = o2;
  }
}

// A fused gather's inputs that do not depend on the launch's own merges, loaded during the merge
// (k_merge_gather): lane f < 55 the query's feature f as K2p reads it (the B' part stale exactly
// at the two step-t pixels of QHand, which the gather substitutes), lane k < 15 the causal
// neighbour k's source pixel and A' image (stale at the same two pixels)
struct QPre {
  bool on = false;
  double v = 0.;
  int sr = 0, sc = 0, si = 0;
  int nn = -1;  // lane 15 + k: causal neighbour k's exact NN row (option "nn_bound")
};
__device__ __forceinline__ QPre qpre_load(const LevelGeo &g, const StepDesc &sn, const Imgs &B, const JobPtrs &jp, int m, int lane) {
  constexpr int D = 55;
  QPre p;
  p.on = true;
  const QPix px = ia_qpix(sn, g.bw, m);
  const int r = px.r, c = px.c;
  if (lane < D) p.v = feat<1>(B, lane, r, c, 0);
  if (px.qi > 0 && lane < 15) {
    const int nr = r - 2 + lane / 5, nc = c - 2 + lane % 5;
    if (nr >= 0 && nc >= 0 && nc < g.bw && nr * g.bw + nc < px.qi) {
      const int nb = nr * g.bw + nc;
      p.sr = jp.s[2 * nb];
      p.sc = jp.s[2 * nb + 1];
      p.si = jp.im[nb];
    }
  }
  if (px.qi > 0 && jp.nn && lane >= 15 && lane < 30) {
    const int k = lane - 15, nr = r - 2 + k / 5, nc = c - 2 + k % 5;
    if (nr >= 0 && nc >= 0 && nc < g.bw && nr * g.bw + nc < px.qi) p.nn = jp.nn[nr * g.bw + nc];
  }
  return p;
}

// U' candidate row of lane (0..14: coherence candidate of causal neighbour lane, 15..29: the
// neighbour's NN row shifted; gather_p_query's sets) from the neighbour's s / im / NN row, -1 when
// it falls outside A or the neighbour has none
__device__ __forceinline__ int ucand_row(const LevelGeo &g, int r, int c, int nr, int nc, bool nnl, int sr, int sc, int si,
                                         int nnrow) {
  if (nnl) {
    sr = -1;
    if (nnrow >= 0 && nnrow < g.NA) {
      const unsigned hw = (unsigned)g.ah * (unsigned)g.aw;
      si = (int)((unsigned)nnrow / hw);
      const unsigned rem = (unsigned)nnrow - (unsigned)si * hw;
      sr = (int)(rem / (unsigned)g.aw);
      sc = (int)(rem - (unsigned)sr * (unsigned)g.aw);
    }
  }
  const int tr = sr + r - nr, tc = sc + c - nc;
  return (sr >= 0 && tr >= 0 && tr < g.ah && tc >= 0 && tc < g.aw) ? (si * g.ah + tr) * g.aw + tc : -1;
}

// K2p's work for one query m of step sd (one wave): q64, qn2, fragments, pruning record (also
// returned, uniform, for the owner-computes publish); xh0 / xh1 (optional) receive the query's
// hi / lo columns
template <int KS, bool IMG, bool FUSE>
__device__ __forceinline__ void gather_p_query(const LevelGeo &g, const StepDesc &sd, const Imgs &B, const JobPtrs &jp, int m,
                                               int lane, const double *__restrict__ mu_part, double *__restrict__ q64,
                                               double *__restrict__ qn2, _Float16 *__restrict__ qf,
                                               const double *__restrict__ db64, const double *__restrict__ basis, double ufac,
                                               float4 *__restrict__ qinfo, const Imgs &A, double *qsh, _Float16 *xh0,
                                               _Float16 *xh1, const QHand &h, float4 &o0, float4 &o1, float4 &o2,
                                               const QPre &pf = QPre{}, unsigned long long *gst = nullptr) {
  constexpr int D = 55, KD = 16 * KS;
#if IA_PROBE & 8
#define IA_GST(k) do { if (gst) { __builtin_amdgcn_s_waitcnt(0); __builtin_amdgcn_sched_barrier(0); \
                       gst[k] = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } } while (0)
#else
#define IA_GST(k) do { (void)gst; } while (0)
#endif
  IA_GST(0);
  static_assert(KD <= IA_WAVE, "one feature per lane");
  const QPix px = ia_qpix(sd, g.bw, m);
  const int32_t *__restrict__ s = jp.s, *__restrict__ im = jp.im;
  const int r = px.r, c = px.c, qi = px.qi;
  // U' candidate of this lane: lanes 0..14 the coherence candidates (product(rows, cols) order as
  // merge_fused); with option "nn_bound" lanes 15..29 the same causal neighbours' exact NN rows,
  // shifted by the neighbour's offset like a coherence candidate.  Any DB row's exact distance
  // bounds the NN distance from above, so U' stays a valid bound whatever row a slot holds (an
  // out-of-range or missing one is skipped); only its tightness depends on them.
  int crow = -1;
  const bool nnl = jp.nn && lane >= 15 && lane < 30;
  if (qi > 0 && (lane < 15 || nnl)) {
    const int k = lane < 15 ? lane : lane - 15;
    const int nr = r - 2 + k / 5, nc = c - 2 + k % 5;
#ifdef IA_EXP_NOABOVE  // experiment: U' without the row-above step-t neighbour's candidates
    const bool skip_above = FUSE && nr == h.r1 && nc == h.c1;
#else
    const bool skip_above = false;
#endif
    if (nr >= 0 && nc >= 0 && nc < g.bw && nr * g.bw + nc < qi && !skip_above) {
      const int nb = nr * g.bw + nc;
      int sr = 0, sc = 0, si = 0, nnrow = -1;
      if (!nnl) {
        if (FUSE && nr == h.r0 && nc == h.c0) {
          sr = h.s0r; sc = h.s0c; si = h.i0;
        } else if (FUSE && nr == h.r1 && nc == h.c1) {
          sr = h.s1r; sc = h.s1c; si = h.i1;
        } else if (pf.on) {
          sr = pf.sr; sc = pf.sc; si = pf.si;
        } else {
          sr = s[2 * nb]; sc = s[2 * nb + 1]; si = im[nb];
        }
      } else {
        nnrow = (FUSE && nr == h.r0 && nc == h.c0) ? h.n0
                : (FUSE && nr == h.r1 && nc == h.c1) ? h.n1
                : pf.on ? pf.nn : jp.nn[nb];
      }
      crow = ucand_row(g, r, c, nr, nc, nnl, sr, sc, si, nnrow);
    }
  }
  double ss = 0., p[IA_NPC];
#pragma unroll
  for (int i = 0; i < IA_NPC; i++) p[i] = 0.;
  if (lane < KD) {
    const int f = lane;
    if (f < D) {
      double v;
      if (pf.on) {  // prefetched; the B' part substituted at the two step-t pixels
        v = pf.v;
        if (FUSE && f >= 43) {
          const int k = f - 43, y = ia_reflect(r + k / 5 - 2, B.h), x = ia_reflect(c + k % 5 - 2, B.w);
          v = (y == h.r0 && x == h.c0) ? h.v0 : (y == h.r1 && x == h.c1) ? h.v1 : v;
        }
      } else {
        v = feat_q1<FUSE>(B, f, r, c, h);
      }
      q64[(int64_t)m * D + f] = v;
      qsh[f] = v;
      const double qc = v - mu_part[feat_part<1>(f)];
      ss = qc * qc;
      put_qh<KS>(qf, m, f, -2.0 * qc);
      if (xh0) split_h(-2.0 * qc, xh0[f], xh1[f]);
#pragma unroll
      for (int i = 0; i < IA_NPC; i++) p[i] = basis[i * D + f] * qc;
    } else {
      put_qh<KS>(qf, m, f, f == D ? IA_NORM_SCALE : 0.);
      if (xh0) split_h(f == D ? IA_NORM_SCALE : 0., xh0[f], xh1[f]);
    }
  }
  IA_GST(1);
  ss = wave_sum_d(ss);
#pragma unroll
  for (int i = 0; i < IA_NPC; i++) p[i] = wave_sum_d_x(p[i]);
  IA_GST(2);
  __builtin_amdgcn_wave_barrier();  // qsh written by this wave's lanes, read below
  double u = DBL_MAX;
  if (crow >= 0) u = exact_dist_level<1>(db64, crow, qsh, IMG ? &A : nullptr);
  u = wave_min_d_x(u);
  IA_GST(3);
  // the pruning record (uniform values): projection interval, U' and the Morton key, and K3p's
  // hi x hi block filter bound (k3p_variant 14/15, ia_k3h.hip k3p_filtered): value bound
  // z >= U' - |q'|^2 with the f32 rounding of z and of the kernel's lim = z + R_t (...)
  // (2^-22 (|q'|^2 + U')) and the subnormal / norm-column terms (2^-24 (16 |q'| + 300));
  // w = 2^-8 |q'| (twice the relative error term's |q'| part)
  const double qn = sqrt(ss);
  const bool fin = u < DBL_MAX;
  const unsigned key = fin ? prune_key(p, basis + IA_NPC * D) : IA_PRUNE_KEY_INF;
  const float up = fin ? round_up_f(u * ufac) : INFINITY;
  const float z = fin ? round_up_f((double)up - ss + 0x1p-22 * (ss + (double)up) + 0x1p-24 * (16.0 * qn + 300.0)) : INFINITY;
  const float w = round_up_f(0x1p-8 * qn * (1.0 + 0x1p-40));
  o0 = make_float4(round_down_f(p[0] - IA_PRUNE_MABS), round_down_f(p[1] - IA_PRUNE_MABS), round_down_f(p[2] - IA_PRUNE_MABS),
                   round_down_f(p[3] - IA_PRUNE_MABS));
  o1 = make_float4(round_up_f(p[0] + IA_PRUNE_MABS), round_up_f(p[1] + IA_PRUNE_MABS), round_up_f(p[2] + IA_PRUNE_MABS),
                   round_up_f(p[3] + IA_PRUNE_MABS));
  o2 = make_float4(up, __uint_as_float(key), z, w);
  if (lane == 0) {
    qn2[m] = ss;
    qinfo[3 * m] = o0;
    qinfo[3 * m + 1] = o1;
    qinfo[3 * m + 2] = o2;
  }
  IA_GST(4);
#undef IA_GST
}

// ------------------------------------------------------------------------------------------
// K2p: K2h for the pruned scan (1 channel) — one wave per query.  Besides the split-f16 query
// fragments it writes the query's pruning record (ia_prune.h), qinfo[3m .. 3m+2]:
//   (qlo_0..3), (qhi_0..3): f32 interval around the fp64 projection onto the level's basis
//   (U', key bits, 0, 0):   U' from the exact fp64 distance of the best coherence candidate
//                           (best_coherence_match's candidate set: the causal 5x5 neighbours'
//                           shifted source pixels, all final at this wavefront step), the
//                           Morton key of the projection (sort order of the query tiles)
// ------------------------------------------------------------------------------------------
template <int KS, bool IMG, class JS>
__global__ void __launch_bounds__(IA_PQ_WG) k_gather_query_p(LevelGeo g, StepDesc sd, Imgs B, JS jobs,
                                                          const double *__restrict__ mu_part,
                                                          double *__restrict__ q64, double *__restrict__ qn2,
                                                          _Float16 *__restrict__ qf, const double *__restrict__ db64,
                                                          const double *__restrict__ basis, double ufac,
                                                          float4 *__restrict__ qinfo, Imgs A, XOPub xp) {
  constexpr int KD = 16 * KS;
  __shared__ double qsh[IA_PQ_WPB][Geo<1>::DS];
  __shared__ __attribute__((aligned(16))) _Float16 xh[IA_PQ_WPB][2][KD];  // owner publish: the query's hi / lo columns
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m = blockIdx.x * IA_PQ_WPB + wv;
  if (m >= sd.Mpad) return;
  float4 i0, i1, i2;
  if (m >= sd.J * sd.M) {
    gather_p_pad<KS>(m, lane, qf, qinfo, i0, i1, i2);
    if (xp.W && lane < KD) xh[wv][0][lane] = xh[wv][1][lane] = (_Float16)0.f;
  } else {
    const QPix px = ia_qpix(sd, g.bw, m);
    const JobPtrs jp = jobs.get(px.job);
    if constexpr (!JS::single) B = job_imgs(B, jp);  // single job: B already holds its images
    gather_p_query<KS, IMG, false>(g, sd, B, jp, m, lane, mu_part, q64, qn2, qf, db64, basis, ufac, qinfo, A, qsh[wv],
                                   xp.W ? xh[wv][0] : nullptr, xh[wv][1], QHand{}, i0, i1, i2);
  }
  if (xp.W) xo_publish<KS>(xp, m, lane, xh[wv][0], xh[wv][1], i0, i1, i2);
}


struct MergeOut {  // one pixel's result: B' value (first channel), source pixel and A' image
  double v;
  int pr, pc, img;
  int nn;  // its certified exact NN row (-1: none)
};

// Fused single-rank merge of query m: certified exact NN + coherence + kappa + writeback.
// Memory is touched in two dependent rounds: (1) the K3 records, the coherence neighbours'
// s/im and the query/weights (staged in LDS), (2) ONE fp64-DB row per lane, in which lane
// k < 15 evaluates coherence candidate k and lanes 15..63 the MFMA candidates worth an exact
// rerank (placed by mbcnt rounds); every lane gets the exact unweighted distance (ranking),
// the weighted one (kappa rule) and its row's A' value (the B' write) from the same round.
// Candidates beyond the 49 rerank lanes (rare) are evaluated by the lanes that listed them.
// Wave reductions use DPP / permlane exchanges (no LDS round trips).
struct NoPre {
  __device__ __forceinline__ void operator()() const {}
};
template <int CH, bool IMG, int RPL, class Pre = NoPre>
__device__ __forceinline__ void merge_fused(const LevelGeo &g, const StepDesc &sd, const Imgs &A, const MergeArgs &a,
                                            int m, const JobPtrs &jp, const QPix &px,
                                            double *qs, double *ws, int *cand_row, float *cand_v,
                                            MergeOut *out = nullptr, Pre pre = Pre{}) {
#if IA_PROBE & 8
  unsigned long long stamp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  IA_STAMP(0);
  // RPL: records per lane (nwg <= 64 RPL); 4 for the split-f16 scans (<= 256 workgroups)
  constexpr int NCOH = 15, NRR = IA_WAVE - NCOH;  // lanes for coherence / rerank candidates
  const int lane = threadIdx.x & 63;
  const int r = px.r, c = px.c, qi = px.qi;
  int32_t *__restrict__ s = jp.s, *__restrict__ im = jp.im;
  double *__restrict__ Bp = jp.Bp;
  const double *__restrict__ weights = jp.weights;
  const double kf = jp.kf;
  const double *q = a.q64 + (int64_t)m * Geo<CH>::D;
  const float4 *rr = a.rec + (int64_t)m * a.nwg;
  const float *rT = a.recT + (int64_t)m * a.nwg;
  const unsigned hw = (unsigned)g.ah * (unsigned)g.aw;

  // ---- round 1: records (clamped, unconditional loads), coherence neighbours, query/weights
  float v1[RPL], v2[RPL], tt[RPL];
  int i1[RPL], i2[RPL];
  int xslot = 0;  // owner-computes sharded step: the query's slot in the step layout
  if (a.xo_W) {
    const int o = m / a.xo_M;
    xslot = a.xo_inv[(a.xo_o0 + o) * a.xo_QTs * IA_TILE + (m - o * a.xo_M)];
  }
#pragma unroll
  for (int j = 0; j < RPL; j++) {
    const int w = min(lane + IA_WAVE * j, a.nwg - 1);
    float4 x;
    float t;
    if (a.xo_W) {  // records pushed by every shard's scan: wait for this step's (T, seq)
      const int64_t ix = (int64_t)w * a.xo_Mrec + xslot;
      const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
      // after an earlier timeout of this context: no waiting (one lost peer costs one timeout)
      const long long lim = __hip_atomic_load(a.xo_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? -1 : a.xo_timeout;
      unsigned long long ts;
      // relaxed: the records are uncached (nothing stale to invalidate; an acquire would
      // invalidate this CU's caches on every poll); the float4 load issues after the seq was seen
      while (((ts = __hip_atomic_load(const_cast<unsigned long long *>(a.xo_rts) + ix, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_SYSTEM)) >> 32) != a.xo_seq) {
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > lim) {
          atomicOr(a.xo_err, 8u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      x = a.rec[ix];
      t = __uint_as_float((unsigned)ts);
    } else {
      x = rr[w];
      t = rT[w];
    }
    const bool ok = lane + IA_WAVE * j < a.nwg;
    v1[j] = ok ? x.x : FLT_MAX;
    v2[j] = ok ? x.z : FLT_MAX;
    tt[j] = ok ? t : FLT_MAX;
    i1[j] = __float_as_int(x.y);
    i2[j] = __float_as_int(x.w);
  }
  for (int f = lane; f < Geo<CH>::D; f += IA_WAVE) {
    qs[f] = q[f];
    ws[f] = weights[f];
  }
  int crow = -1, cpr = -1, cpc = -1, cim = 0;
  if (qi > 0 && lane < NCOH) {  // best_coherence_match candidates, product(rows, cols) order
    const int nr = r - 2 + lane / 5, nc = c - 2 + lane % 5;
    if (nr >= 0 && nc >= 0 && nc < g.bw && nr * g.bw + nc < qi) {
      const int nb = nr * g.bw + nc;
      const int tr = s[2 * nb] + r - nr, tc = s[2 * nb + 1] + c - nc;
      const int ti = im[nb];
      if (tr >= 0 && tr < g.ah && tc >= 0 && tc < g.aw) {
        cpr = tr;
        cpc = tc;
        cim = ti;
        crow = (ti * g.ah + tr) * g.aw + tc;
      }
    }
  }
  const double R = (double)__uint_as_float(*a.Rbits);
  const double qn2 = a.qn2[m];
#if IA_PROBE & 8
  if (v1[0] == 12345.f && crow == 7) stamp[7] = 1;  // force round 1 to land here
#endif
  IA_STAMP(1);

  // ---- MFMA candidates that may be the exact winner -> lanes 15..63 (mbcnt placement rounds)
  float a1 = FLT_MAX;
#pragma unroll
  for (int j = 0; j < RPL; j++) a1 = fminf(a1, v1[j]);
  a1 = wave_min_f_x(a1);
  const double qn = sqrt(qn2);
  const double eps = merge_eps(a, R, qn);
  const double thr = (double)a1 + 2.0 * eps;
  unsigned cmask = 0;
  // a float v satisfies v <= thr exactly when v <= thr rounded down to float: one conversion
  // instead of one per compared value
  const float thf = round_down_f(thr);
#pragma unroll
  for (int j = 0; j < RPL; j++) {
    if (v1[j] <= thf && i1[j] >= 0 && i1[j] < a.NA) cmask |= 1u << (2 * j);
    if (v2[j] <= thf && i2[j] >= 0 && i2[j] < a.NA) cmask |= 1u << (2 * j + 1);
  }
  int placed = 0;  // candidates given a rerank lane so far (wave-uniform)
  unsigned long long bal = __ballot(cmask != 0);
  while (bal && placed < NRR) {
    const int pos = placed + lane_prefix(bal);
    if (cmask != 0 && pos < NRR) {
      float v;
      cand_row[pos] = lowest_cand<RPL>(cmask, i1, i2, v1, v2, v);
      cand_v[pos] = v;
      cmask &= cmask - 1;
    }
    placed += __popcll(bal);
    bal = __ballot(cmask != 0);
  }
  const int n_cand = min(placed, NRR);
  __builtin_amdgcn_wave_barrier();
  int my_row = lane < NCOH ? crow : (lane - NCOH < n_cand ? cand_row[lane - NCOH] : -1);
  const float my_v = lane >= NCOH && my_row >= 0 ? cand_v[lane - NCOH] : FLT_MAX;
  IA_STAMP(2);
  // (k_merge_gather: the next query's step-independent inputs are loaded here, in flight together
  // with round 2's rows instead of after them)
  pre();

  // ---- round 2: one fp64-DB row + its A' value per lane
  double unw = DBL_MAX, wsq = 0.;
  double av[CH];
#pragma unroll
  for (int k = 0; k < CH; k++) av[k] = 0.;
  if (my_row >= 0) {
    const unsigned img = (unsigned)my_row / hw;
    const double *src = A.p3 + img * A.img_stride_f + (int64_t)((unsigned)my_row - img * hw) * CH;
#pragma unroll
    for (int k = 0; k < CH; k++) av[k] = src[k];
    row_dists<CH>(a.db64, my_row, qs, ws, unw, wsq, IMG ? &A : nullptr);
  }
  // bound audit: the exact distance of every reranked candidate must lie within eps of its
  // MFMA value + |q'|^2 (a violation would void the certification; counted, never expected)
  const bool viol = lane >= NCOH && my_row >= 0 && fabs(unw - qn2 - (double)my_v) > eps;
  const bool any_viol = __ballot(viol) != 0;
#if IA_PROBE & 8
  if (unw == 12345.) stamp[7] = 2;
#endif
  IA_STAMP(3);

  // exact NN candidates of this lane: its rerank row, then any overflow it listed (rare)
  double nd = (lane >= NCOH && my_row >= 0) ? unw : DBL_MAX;
  int ni = (lane >= NCOH && my_row >= 0) ? my_row : INT_MAX;
  bool recompute_app = false;
  int n_over = 0;
  while (cmask) {
    float v;
    const int row = lowest_cand<RPL>(cmask, i1, i2, v1, v2, v);
    cmask &= cmask - 1;
    double u, wq;
    row_dists<CH>(a.db64, row, qs, ws, u, wq, IMG ? &A : nullptr);
    if (u < nd || (u == nd && row < ni)) {
      nd = u;
      ni = row;
    }
    n_over++;
  }
  if (__ballot(n_over > 0)) recompute_app = true;
  // NN winner (lowest index on ties) and coherence winner (first argmin of the norm): the two
  // minima by interleaved DPP butterflies, then the lanes that hold them by ballot (a tie in the
  // NN distance between lanes - exact duplicate rows - takes the lowest row by a third butterfly)
  const double dkl = (lane < NCOH && my_row >= 0) ? cr_sqrt(unw) : DBL_MAX;
  const double bd0 = wave_min_d_x(nd), dk = wave_min_d_x(dkl);
  double bd = bd0;
  int bi = INT_MAX;
  if (bd0 < DBL_MAX) {
    const unsigned long long eqn = __ballot(nd == bd0);
    bi = __builtin_amdgcn_readlane(ni, __ffsll((long long)eqn) - 1);
    if (eqn & (eqn - 1)) {  // (wave-uniform, rare) several lanes at the same distance
      int x = nd == bd0 ? ni : INT_MAX;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o, 64));
      bi = x;
    }
  }
  const int kk = dk < DBL_MAX ? __ffsll((long long)__ballot(dkl == dk)) - 1 : INT_MAX;
  const unsigned long long own = __ballot(lane >= NCOH && my_row >= 0 && my_row == bi && unw == bd);
  double wsq_app = 0.;
  int app_lane = 0;
  if (own) {
    app_lane = __ffsll((long long)own) - 1;
    wsq_app = readlane_d(wsq, app_lane);
  } else {
    recompute_app = true;
  }
  IA_STAMP(4);

  // certification (see certified_winner): rescan chunks whose threshold does not clear bd
  const double theta = cert_theta(a, R, qn, qn2, bd);
  const float thetaf = round_down_f(theta);  // (t <= theta  <=>  t <= theta rounded down, t a float)
  unsigned long long nfb = 0;
#pragma unroll
  for (int jb = 0; jb < RPL; jb++) {
    unsigned long long mask = __ballot(tt[jb] <= thetaf);
    while (mask) {
      const int j = __ffsll((long long)mask) - 1;
      mask &= mask - 1;
      const int wgid = jb * IA_WAVE + j;
      double cd = DBL_MAX;
      int ci = INT_MAX;
      if (a.rr) {
        // pruned scan: chunk = tiles wgid, wgid + nwg, ...  Only rows with exact distance <= bd
        // can displace the winner, and such a row's tile has a projection lower bound
        // <= bd * ufac (ia_prune.h), so the rescan visits just the tiles that pass that box
        // test (one tile per lane), two tiles per wave pass
        const float4 ql = a.qinfo[3 * m], qh = a.qinfo[3 * m + 1];
        const float ub = round_up_f(bd * a.ufac);
        // the chunk's tiles t0 + tst k < tend (owner-computes step: chunk wgid mod nch of shard
        // wgid / nch, in that shard's storage range of the whole level's table)
        int64_t t0 = wgid, tst = a.nwg, tend = a.NT;
        if (a.xo_W) {
          const int sh = wgid / a.xo_nch;
          t0 = ia_shard_off(a.NT, a.xo_W, sh) + (wgid - sh * a.xo_nch);
          tst = a.xo_nch;
          tend = ia_shard_off(a.NT, a.xo_W, sh + 1);
        }
        for (int64_t tb = 0; t0 + tst * tb < tend; tb += IA_WAVE) {
          const int64_t t = t0 + tst * (tb + lane);
          bool nd = false;
          if (t < tend) nd = prune_lb(a.boxes[2 * t], a.boxes[2 * t + 1], ql, qh) <= ub;
          unsigned long long nm = __ballot(nd);
          while (nm) {
            const int j0 = __ffsll((long long)nm) - 1;
            nm &= nm - 1;
            int j1 = -1;
            if (nm) {
              j1 = __ffsll((long long)nm) - 1;
              nm &= nm - 1;
            }
            const int j = lane < 32 ? j0 : j1;
            if (j >= 0) {
              const int64_t i = a.pos2row[(t0 + tst * (tb + j)) * IA_TILE + (lane & 31)];
              if (i < a.NA) {
                const double d = exact_dist_level<CH>(a.db64, i, qs, IMG ? &A : nullptr);
                if (d < cd || (d == cd && (int)i < ci)) { cd = d; ci = (int)i; }
              }
            }
          }
        }
      } else {
        const int64_t p0 = (int64_t)a.pos0 + (int64_t)wgid * a.tpw * IA_TILE;
        const int64_t p1 = min((int64_t)a.pos_end, p0 + (int64_t)a.tpw * IA_TILE);
        for (int64_t p = p0 + lane; p < p1; p += IA_WAVE) {
          const int64_t i = ia_pos_row_t(p, a.NT, a.pos2row);
          if (i >= a.NA) continue;
          const double d = exact_dist_level<CH>(a.db64, i, qs, IMG ? &A : nullptr);
          if (d < cd || (d == cd && (int)i < ci)) { cd = d; ci = (int)i; }
        }
      }
      double du = DBL_MAX;
      int iu = INT_MAX;
      wave_min2_di(cd, ci, du, iu);
      (void)du;
      (void)iu;
      if (cd < bd || (cd == bd && ci < bi)) {
        bd = cd;
        bi = ci;
        recompute_app = true;
      }
      nfb++;
    }
  }
  IA_STAMP(5);

  int img = (int)((unsigned)bi / hw);
  const unsigned rem = (unsigned)bi - (unsigned)img * hw;
  int pr = (int)(rem / (unsigned)g.aw), pc = (int)(rem - (unsigned)pr * (unsigned)g.aw);
  const int app_img = img, app_pr = pr, app_pc = pc;
  double dbg_app = 0., dbg_coh = 0.;
  bool kamb = false;
  bool coh_won = false;
  int src_lane = recompute_app ? -1 : app_lane;  // lane holding the chosen row's A' value
  if (kk != INT_MAX) {  // a coherence candidate exists (never for the level's first pixel)
    // (ds_bpermute here: v_readlane at kk measured 0.25 us slower per launch, profiles/r06/trims)
    const int kpr = __shfl(cpr, kk, 64), kpc = __shfl(cpc, kk, 64), kim = __shfl(cim, kk, 64);
    const double wsq_coh = __shfl(wsq, kk, 64);
    if (recompute_app) {
      double u, wq = 0.;
      if (lane == 0) row_dists<CH>(a.db64, bi, qs, ws, u, wq, IMG ? &A : nullptr);
      wsq_app = readlane_d(wq, 0);
    }
    // compute_distance = norm(x)**2 = sqrt(sum x^2)**2 ; kappa rule image_analogies.py:206
    const double y_app = cr_sqrt(wsq_app), y_coh = cr_sqrt(wsq_coh);
    const double d_app = y_app * y_app, d_coh = y_coh * y_coh;
    kamb = kappa_ambiguous(y_app, d_app, y_coh, d_coh, kf);
    dbg_app = wsq_app;  // the host finishes compute_distance as np.sqrt(v) ** 2 (libm pow)
    dbg_coh = wsq_coh;
    if (d_coh <= d_app * kf) {
      img = kim;
      pr = kpr;
      pc = kpc;
      coh_won = true;
      src_lane = kk;
    }
  }
  IA_STAMP(6);
  double val[CH];
#pragma unroll
  for (int k = 0; k < CH; k++) val[k] = src_lane >= 0 ? readlane_d(av[k], src_lane) : 0.;
  if (src_lane < 0) {  // winner from an overflow candidate or a rescan: fetch its A' value
#pragma unroll
    for (int k = 0; k < CH; k++) val[k] = A.p3[img * A.img_stride_f + ((int64_t)pr * g.aw + pc) * CH + k];
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < CH; k++) Bp[(int64_t)qi * CH + k] = val[k];
    s[2 * qi] = pr;
    s[2 * qi + 1] = pc;
    im[qi] = img;
    if (jp.nn) jp.nn[qi] = bi >= 0 && bi < a.NA ? bi : -1;  // option "nn_bound"
    // per-pixel stats word (no shared-counter atomics: hundreds of waves adding to one
    // address serialise at L2 and dominated this kernel); reduced once per level
    const int slot = placed + 0;
    jp.pstat[qi] = (unsigned)min(slot, 0xffff) | ((unsigned)min((int)nfb, 0x1fff) << 16) | (kamb ? 1u << 29 : 0u) |
                  (coh_won ? 1u << 30 : 0u) |
                  (any_viol ? 1u << 31 : 0u);
    if (jp.dbg_src) {  // debug=True structures (image_analogies.py:224-240): p_app, r_star, d_app, d_coh
      const bool has_coh = kk != INT_MAX;
      int32_t *o = jp.dbg_src + (int64_t)qi * 6;
      o[0] = app_pr;
      o[1] = app_pc;
      o[2] = app_img;
      o[3] = has_coh ? r - 2 + kk / 5 : 0;
      o[4] = has_coh ? c - 2 + kk % 5 : 0;
      o[5] = has_coh ? 1 : 0;
      jp.dbg_dist[2 * qi] = dbg_app;
      jp.dbg_dist[2 * qi + 1] = dbg_coh;
    }
  }
  if (out) {  // the pixel's result (wave-uniform) for a fused next-step gather (k_merge_gather)
    out->v = val[0];
    out->pr = pr;
    out->pc = pc;
    out->img = img;
    out->nn = bi >= 0 && bi < a.NA ? bi : -1;
  }
#if IA_PROBE & 8
  if (lane == 0 && m == sd.M / 2 && (sd.t % 256) == 128) {
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t7 = __builtin_amdgcn_s_memtime();
    printf("STAMP bw=%d t=%d M=%d slot=%d nfb=%d d1=%llu d2=%llu d3=%llu d4=%llu d5=%llu d6=%llu d7=%llu\n", g.bw, sd.t,
           sd.M, placed, (int)nfb, stamp[1] - stamp[0], stamp[2] - stamp[1], stamp[3] - stamp[2], stamp[4] - stamp[3],
           stamp[5] - stamp[4], stamp[6] - stamp[5], t7 - stamp[6]);
  }
#endif
}

template <int CH, bool FUSED, bool IMG, class JS, int RPL = IA_WG_TARGET / IA_WAVE>
__global__ void __launch_bounds__(IA_PQ_WG) k_merge_level(LevelGeo g, StepDesc sd, Imgs A, MergeArgs ma, Winner *__restrict__ win,
                                                        JS jobs) {
  const int m = __builtin_amdgcn_readfirstlane(blockIdx.x * IA_PQ_WPB + (threadIdx.x >> 6));  // wave-uniform
  if (m >= sd.J * sd.M) return;
  const QPix px = ia_qpix(sd, g.bw, m);
  const JobPtrs jp = jobs.get(px.job);
  if constexpr (FUSED) {
    __shared__ double qsh[IA_PQ_WPB][Geo<CH>::DS], wsh[IA_PQ_WPB][Geo<CH>::DS];
    __shared__ int crsh[IA_PQ_WPB][IA_WAVE];
    __shared__ float cvsh[IA_PQ_WPB][IA_WAVE];
    const int wv = threadIdx.x >> 6;
    const unsigned long long t0 = ma.stamp ? ia_clock() : 0ull;  // option "stamps"
    merge_fused<CH, IMG, RPL>(g, sd, A, ma, m, jp, px, qsh[wv], wsh[wv], crsh[wv], cvsh[wv]);
    if (ma.stamp && (threadIdx.x & 63) == 0) ia_stamp_wg(ma.stamp, t0);
    return;
  }
  const double *q = ma.q64 + (int64_t)m * Geo<CH>::D;
  unsigned stat = 0;
  const Winner wn = certified_winner(ma, m, [&](int64_t row) {
    return exact_dist_level<CH>(ma.db64, row, q, IMG ? &A : nullptr);
  }, &stat);
  if constexpr (FUSED) {
    finish_pixel<CH>(g, A, ma.db64, px.r, px.c, wn.idx, q, jp.s, jp.im, jp.Bp, jp.weights, jp.kf, jp.pstat, stat, jp.nn);
  } else {
    if ((threadIdx.x & 63) == 0) {
      win[m] = wn;
      if (jp.pstat) jp.pstat[px.qi] = stat;  // finish adds the coherence bit
    }
  }
}

// ------------------------------------------------------------------------------------------
// K4 + K2p fused (option "fuse_gather"): K4 of step t, then K2p of step t + 1, one launch.
// Pixel (r, c + 1) of step t + 1 reads two results of step t: its own row's (r, c) and the row
// above's (r - 1, c + 3) (skew 3: both lie on step t); everything else it reads is older.  So
// wave w (query w of step t, row r = r0 + w) merges (r, c), hands its result to row r + 1
// through an uncached slot (fields, store completion, then the step's seq), and gathers
// (r, c + 1), waiting for the slot of row r - 1: a wave of the same launch with a LOWER index
// (rows ascend with the query index), dispatched before it, so the waits always drain.  Wave
// M gathers the row entering at step t + 1 (column 0; its row above is wave M - 1), the waves
// after it the step's pad queries.  The query buffers alternate by step parity (this launch's
// merge reads step t's half while its gathers write step t + 1's).
// ------------------------------------------------------------------------------------------
// K2h's work for one query m of step sd (unpruned split-f16 levels), with the fused gather's
// two step-t pixels substituted (QHand) in the B' part
template <int KS>
__device__ __forceinline__ void gather_h_query_fused(const LevelGeo &g, const StepDesc &sd, const Imgs &B, int m, int lane,
                                                     const double *__restrict__ mu_part, double *__restrict__ q64,
                                                     double *__restrict__ qn2, _Float16 *__restrict__ qf, const QHand &h) {
  constexpr int D = 55, KD = 16 * KS;
  static_assert(KD <= IA_WAVE, "one feature per lane");
  const QPix px = ia_qpix(sd, g.bw, m);
  const int r = px.r, c = px.c;
  double ss = 0.;
  if (lane < KD) {
    const int f = lane;
    if (f < D) {
      double v;
      if (f >= 43) {  // the B' part (causal 5x5 at (r, c), k < 12)
        const int k = f - 43, y = ia_reflect(r + k / 5 - 2, B.h), x = ia_reflect(c + k % 5 - 2, B.w);
        v = (y == h.r0 && x == h.c0) ? h.v0 : (y == h.r1 && x == h.c1) ? h.v1 : B.p3[(int64_t)y * B.w + x];
      } else {
        v = feat<1>(B, f, r, c, 0);
      }
      q64[(int64_t)m * D + f] = v;
      const double qc = v - mu_part[feat_part<1>(f)];
      ss = qc * qc;
      put_qh<KS>(qf, m, f, -2.0 * qc);
    } else {
      put_qh<KS>(qf, m, f, f == D ? IA_NORM_SCALE : 0.);
    }
  }
  ss = wave_sum_d(ss);
  if (lane == 0) qn2[m] = ss;
}

// Per-level constants of the fused gather (lane f < 55: its feature's basis column and part mean;
// the key scale), loaded at wave start so no dependent load of them sits behind the handoff.
struct QConst {
  double bas[IA_NPC] = {0., 0., 0., 0.};
  double mu = 0.;
  double sc[IA_NPC] = {0., 0., 0., 0.};
};
__device__ __forceinline__ QConst qconst_load(const NextStep &nx, int lane) {
  constexpr int D = 55;
  QConst k;
  if (lane < D) {
#pragma unroll
    for (int i = 0; i < IA_NPC; i++) k.bas[i] = nx.basis[i * D + lane];
    k.mu = nx.mu[feat_part<1>(lane)];
  }
#pragma unroll
  for (int i = 0; i < IA_NPC; i++) k.sc[i] = nx.basis[IA_NPC * D + i];
  return k;
}

// The fused gather of query mn (step t + 1) for a merge wave of a one-rank pruned level (option
// "prefetch_next"; no publish): everything that does not depend on the row above's step-t result
// runs BEFORE the wait for its handoff - the query's other 54 features (q64, split-f16 fragments,
// projections, |q'|^2 as sums over those lanes) and U': the exact distance of each candidate row
// over those features, the rows requested first so their loads are in flight during the feature
// work.  After the handoff only the late feature (the row above's pixel (r - 1, c + 2) of the
// query's window) is added to each sum.  U' skips the row above's own two candidates (its source
// pixel and NN row, shifted): any DB row's exact distance bounds the NN distance from above, so U'
// stays a valid bound (the scan's passing tiles 0.144 -> 0.147); the summation
// orders of U', |q'|^2 and the projections differ from K2p's, which the bounds' margins cover
// (the NN decisions are the merge's fp64 reranks, unchanged).
template <int KS>
__device__ __forceinline__ void gather_p_early(const LevelGeo &g, const NextStep &nx, const Imgs &B, const JobPtrs &jp,
                                               int job, int mn, int lane, const double *__restrict__ db64, double *qsh,
                                               const QHand &h0, const QPre &pf, const QConst &qk) {
  constexpr int D = 55, KD = 16 * KS, DS = Geo<1>::DS;
  static_assert(KD <= IA_WAVE, "one feature per lane");
#if IA_PROBE & 8
  unsigned long long gst[7] = {__builtin_amdgcn_s_memtime(), 0, 0, 0, 0, 0, 0};
  const bool gprobe = mn == nx.sn.M / 2 && (nx.sn.t % 256) == 129;
#define IA_GST2(k) do { if (gprobe) { __builtin_amdgcn_s_waitcnt(0); __builtin_amdgcn_sched_barrier(0); \
                        gst[k] = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } } while (0)
#else
#define IA_GST2(k) do { } while (0)
#endif
  const StepDesc &sn = nx.sn;
  const QPix pn = ia_qpix(sn, g.bw, mn);
  const int r = pn.r, c = pn.c, qi = pn.qi;
  // the row above's step-t pixel: its result arrives through the handoff slot of row r - 1
  const bool above = r >= 1 && c + 2 < g.bw;
  const int ar = r - 1, ac = c + 2;
  // ---- features (lane f < 55): the prefetched value, this wave's own result substituted
  double v = 0.;
  bool late = false;
  if (lane < D) {
    v = pf.v;
    if (lane >= 43) {
      const int k = lane - 43, y = ia_reflect(r + k / 5 - 2, B.h), x = ia_reflect(c + k % 5 - 2, B.w);
      if (y == h0.r0 && x == h0.c0) v = h0.v0;
      late = above && y == ar && x == ac;
    }
  }
  // (the late pixel can fill several window slots where the window is reflected at the image's
  // top or sides: up to four of the twelve B' slots 43..54)
  const unsigned long long lm = __ballot(late);
  // ---- U' candidate rows: lanes 0..14 the causal neighbours' shifted sources, 15..29 (option
  // "nn_bound") their shifted NN rows; the row above's pixel skipped (its result is late)
  int crow = -1;
  const bool nnl = jp.nn && lane >= 15 && lane < 30;
  if (qi > 0 && (lane < 15 || nnl)) {
    const int k = lane < 15 ? lane : lane - 15;
    const int nr = r - 2 + k / 5, nc = c - 2 + k % 5;
    if (nr >= 0 && nc >= 0 && nc < g.bw && nr * g.bw + nc < qi && !(above && nr == ar && nc == ac)) {
      const bool own = nr == h0.r0 && nc == h0.c0;
      const int sr = own ? h0.s0r : pf.sr, sc = own ? h0.s0c : pf.sc, si = own ? h0.i0 : pf.si;
      const int nnrow = own ? h0.n0 : pf.nn;
      crow = ucand_row(g, r, c, nr, nc, nnl, sr, sc, si, nnrow);
    }
  }
  // the candidate row, requested now (in flight during the feature work below)
  double2 rowv[DS / 2];
  {
    const double2 *src = reinterpret_cast<const double2 *>(db64 + (int64_t)(crow >= 0 ? crow : 0) * DS);
#pragma unroll
    for (int i = 0; i < DS / 2; i++) rowv[i] = src[i];
  }
  if (lane < D) qsh[lane] = late ? 0. : v;
  // ---- the non-late features: q64, fragments, projections, |q'|^2 (late lanes hold 0)
  double ss = 0., p[IA_NPC] = {0., 0., 0., 0.}, qc = 0.;
  if (lane < KD) {
    if (lane < D) {
      if (!late) {
        nx.q64[(int64_t)mn * D + lane] = v;
        qc = v - qk.mu;
        ss = qc * qc;
        put_qh<KS>((_Float16 *)nx.qf, mn, lane, -2.0 * qc);
#pragma unroll
        for (int i = 0; i < IA_NPC; i++) p[i] = qk.bas[i] * qc;
      }
    } else {
      put_qh<KS>((_Float16 *)nx.qf, mn, lane, lane == D ? IA_NORM_SCALE : 0.);
    }
  }
  ss = wave_sum_d_x(ss);
#pragma unroll
  for (int i = 0; i < IA_NPC; i++) p[i] = wave_sum_d_x(p[i]);
  IA_GST2(1);
  __builtin_amdgcn_wave_barrier();  // qsh written by this wave's lanes, read below
  // ---- U' partial distances over the non-late features (pairwise order; a late feature adds 0)
  const double *rv = reinterpret_cast<const double *>(rowv);
  double part = pw_sum<D>([&](int f) {
    const double d = rv[f] - qsh[f];
    return ((lm >> f) & 1ull) ? 0. : d * d;
  });
  double al[12];  // the row's values at the B' slots (read after the handoff for the late ones)
#pragma unroll
  for (int k = 0; k < 12; k++) al[k] = rv[43 + k];
  IA_GST2(2);
  // ---- the row above's result (handoff)
  QHand h = h0;
  if (above) {
    const HandSlot *hs = nx.hand + (int64_t)job * g.bh + ar;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(&hs->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != nx.seq) {
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > nx.timeout_ticks) {
        atomicOr(nx.err, 16u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    h.v1 = hs->v;
  }
  IA_GST2(3);
  // ---- the late slots: their value, fragments and terms, in slot order
  if (lm) {
    if (late) {
      nx.q64[(int64_t)mn * D + lane] = h.v1;
      qc = h.v1 - qk.mu;
      put_qh<KS>((_Float16 *)nx.qf, mn, lane, -2.0 * qc);
    }
#pragma unroll
    for (int k = 0; k < 12; k++) {
      if ((lm >> (43 + k)) & 1ull) {  // wave-uniform
        const double qcl = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(qc), 43 + k),
                                            __builtin_amdgcn_readlane(__double2loint(qc), 43 + k));
        ss += qcl * qcl;
#pragma unroll
        for (int i = 0; i < IA_NPC; i++) {
          const double bl = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(qk.bas[i]), 43 + k),
                                             __builtin_amdgcn_readlane(__double2loint(qk.bas[i]), 43 + k));
          p[i] += bl * qcl;
        }
        const double d = al[k] - h.v1;
        part += d * d;
      }
    }
  }
  double u = crow >= 0 ? part : DBL_MAX;
  u = wave_min_d_x(u);
  IA_GST2(4);
  // ---- the pruning record (gather_p_query's, from these sums)
  const double qn = sqrt(ss);
  const bool fin = u < DBL_MAX;
  const unsigned key = fin ? prune_key(p, qk.sc) : IA_PRUNE_KEY_INF;
  const float up = fin ? round_up_f(u * nx.ufac) : INFINITY;
  const float z = fin ? round_up_f((double)up - ss + 0x1p-22 * (ss + (double)up) + 0x1p-24 * (16.0 * qn + 300.0)) : INFINITY;
  const float w = round_up_f(0x1p-8 * qn * (1.0 + 0x1p-40));
  if (lane == 0) {
    nx.qn2[mn] = ss;
    nx.qinfo[3 * mn] = make_float4(round_down_f(p[0] - IA_PRUNE_MABS), round_down_f(p[1] - IA_PRUNE_MABS),
                                   round_down_f(p[2] - IA_PRUNE_MABS), round_down_f(p[3] - IA_PRUNE_MABS));
    nx.qinfo[3 * mn + 1] = make_float4(round_up_f(p[0] + IA_PRUNE_MABS), round_up_f(p[1] + IA_PRUNE_MABS),
                                       round_up_f(p[2] + IA_PRUNE_MABS), round_up_f(p[3] + IA_PRUNE_MABS));
    nx.qinfo[3 * mn + 2] = make_float4(up, __uint_as_float(key), z, w);
  }
  IA_GST2(5);
#if IA_PROBE & 8
  if (gprobe && lane == 0)
    printf("ESTAMP bw=%d t=%d M=%d pre=%llu part=%llu handoff=%llu late=%llu rec=%llu\n", g.bw, sn.t, sn.M, gst[1] - gst[0],
           gst[2] - gst[1], gst[3] - gst[2], gst[4] - gst[3], gst[5] - gst[4]);
#endif
#undef IA_GST2
}

// ------------------------------------------------------------------------------------------
// K4 + K2 fused (option "fuse_gather"): K4 of step t, then the gather (K2p on pruned levels,
// K2h on the others) of step t + 1, one launch.  Pixel (r, c + 1) of step t + 1 reads two
// results of step t: its own row's (r, c) and the row above's (r - 1, c + 3) (skew 3: both lie
// on step t); everything else it reads is older.  So the wave of query (job j, row r) merges
// (r, c), hands its result to row r + 1 through an uncached slot (fields, store completion, then
// the step's seq), and gathers (r, c + 1), waiting for the slot of row r - 1: a wave of the same
// launch with a LOWER index (rows ascend with the query index within a job), dispatched before
// it, so the waits always drain.  Waves J M .. J M + J - 1 gather each job's row entering at
// step t + 1 (column 0; its row above is that job's last merge wave), the waves after them the
// step's pad queries (and, owner-computes ranks with xo_wait, one waiter).  The query buffers
// alternate by step parity (this launch's merges read step t's half while its gathers write
// step t + 1's).
// ------------------------------------------------------------------------------------------
template <int RPL, bool PR, bool XO, class JS>
__device__ __forceinline__ void merge_gather_body(const LevelGeo &g, const StepDesc &sd, const Imgs &A, const MergeArgs &ma,
                                                  const JS &jobs, Imgs B, const NextStep &nx) {
  constexpr int KS = 4;
  const int w = __builtin_amdgcn_readfirstlane(blockIdx.x * IA_PQ_WPB + (threadIdx.x >> 6));
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int J = JS::single ? 1 : sd.J, JM = J * sd.M;
  __shared__ double qsh[IA_PQ_WPB][Geo<1>::DS], wsh[IA_PQ_WPB][Geo<1>::DS];
  __shared__ int crsh[IA_PQ_WPB][IA_WAVE];
  __shared__ float cvsh[IA_PQ_WPB][IA_WAVE];
  __shared__ __attribute__((aligned(16))) _Float16 xh[IA_PQ_WPB][2][16 * KS];  // owner publish: hi / lo columns
  if (XO && w >= JM + J + (nx.sn.Mpad - J * nx.sn.M)) {  // the waiter (nx.wait_n > 0 only)
    // after an earlier timeout of this context: no waiting (one lost peer costs one timeout)
    if (__hip_atomic_load(nx.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    for (int i = lane; i < nx.wait_n; i += IA_WAVE)
      while (__hip_atomic_load(nx.wait_seq + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != nx.xp.seq) {
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > nx.timeout_ticks) {
          atomicOr(nx.err, 4u);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    return;
  }
  QHand h;
  int mn = -1;   // this wave's query of step t + 1
  int job = 0;
  QPre pf;       // its step-independent inputs, prefetched during the merge (pruned levels)
  // the early gather path (gather_p_early): merge waves of one-rank pruned levels, no publish
  const bool early = PR && !XO && !nx.kslot && nx.prefetch && nx.early;
  QConst qk;
  if (early) qk = qconst_load(nx, lane);
#if IA_PROBE & 8  // diagnostic build only: fused merge + gather phase stamps of one sampled wave
  unsigned long long gs[5] = {__builtin_amdgcn_s_memtime(), 0, 0, 0, 0}, gst[5] = {0, 0, 0, 0, 0};
  const bool gprobe = w == sd.M / 2 && (sd.t % 256) == 128 && JM == sd.M;
#endif
  if (w < JM) {
    const QPix px = ia_qpix(sd, g.bw, w);
    job = px.job;
    const JobPtrs jp = jobs.get(job);
    MergeOut o;
    if (px.c + 1 < g.bw) mn = job * nx.sn.M + (px.r - nx.sn.r0);
    const Imgs Bj = JS::single ? B : job_imgs(B, jp);
    auto pre = [&]() {
      if (PR && nx.prefetch && mn >= 0) pf = qpre_load(g, nx.sn, Bj, jp, mn, lane);
    };
    merge_fused<1, false, RPL>(g, sd, A, ma, w, jp, px, qsh[wv], wsh[wv], crsh[wv], cvsh[wv], &o, pre);
    if (px.r + 1 < g.bh && px.c >= 2) {  // row r + 1 gathers (r + 1, c - 2) at step t + 1
      HandSlot *hs = nx.hand + (int64_t)job * g.bh + px.r;
      if (lane == 0) {
        hs->v = o.v;
        hs->sr = o.pr;
        hs->sc = o.pc;
        hs->im = o.img;
        hs->nn = o.nn;
      }
      ia_stores_done();
      if (lane == 0) __hip_atomic_store(&hs->seq, nx.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    h.r0 = px.r;
    h.c0 = px.c;
    h.v0 = o.v;
    h.s0r = o.pr;
    h.s0c = o.pc;
    h.i0 = o.img;
    h.n0 = o.nn;
#if IA_PROBE & 8
    __builtin_amdgcn_s_waitcnt(0);
    gs[1] = __builtin_amdgcn_s_memtime();
#endif
  } else if (w < JM + J) {
    job = w - JM;
    if (nx.sn.t - 3 * (nx.sn.r0 + nx.sn.M - 1) == 0) mn = job * nx.sn.M + nx.sn.M - 1;  // a row enters at column 0
  } else {
    mn = J * nx.sn.M + (w - JM - J);
  }
  if (mn < 0 || mn >= nx.sn.Mpad) return;
  _Float16 *qf = (_Float16 *)nx.qf;
  float4 o0, o1, o2;
  if (mn >= J * nx.sn.M) {
    if constexpr (PR) {
      gather_p_pad<KS>(mn, lane, qf, nx.qinfo, o0, o1, o2);
      if ((XO && nx.xp.W) || (!XO && nx.kslot)) {
        if (lane < 16 * KS) xh[wv][0][lane] = xh[wv][1][lane] = (_Float16)0.f;
        if (XO) xo_publish<KS>(nx.xp, mn, lane, xh[wv][0], xh[wv][1], o0, o1, o2);
        else sorted_publish<KS>(nx, mn, lane, xh[wv][0], xh[wv][1], o0, o1, o2);
      }
    } else {
      if (lane < 16 * KS) put_qh<KS>(qf, mn, lane, 0.);
    }
    return;
  }
  const JobPtrs jp = jobs.get(job);
  if constexpr (!JS::single) B = job_imgs(B, jp);  // single job: B already holds its images
  if constexpr (PR) {
    if (early && pf.on) {
      __builtin_amdgcn_wave_barrier();  // the merge's LDS rows are done with
      gather_p_early<KS>(g, nx, B, jp, job, mn, lane, ma.db64, qsh[wv], h, pf, qk);
      return;
    }
  }
  const QPix pn = ia_qpix(nx.sn, g.bw, mn);
  if (pn.r >= 1 && pn.c + 2 < g.bw) {  // (r - 1, c + 2) of step t: the row above's handoff
    const HandSlot *hs = nx.hand + (int64_t)job * g.bh + (pn.r - 1);
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    // relaxed: the slot is uncached (nothing stale to invalidate); its fields load after the
    // seq was seen
    while (__hip_atomic_load(&hs->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != nx.seq) {
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > nx.timeout_ticks) {
        atomicOr(nx.err, 16u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    h.r1 = pn.r - 1;
    h.c1 = pn.c + 2;
    h.v1 = hs->v;
    h.s1r = hs->sr;
    h.s1c = hs->sc;
    h.i1 = hs->im;
    h.n1 = hs->nn;
  }
#if IA_PROBE & 8
  __builtin_amdgcn_s_waitcnt(0);
  gs[2] = __builtin_amdgcn_s_memtime();
#endif
  __builtin_amdgcn_wave_barrier();  // the merge's LDS rows are done with
  if constexpr (PR) {
    const bool pub = (XO && nx.xp.W) || (!XO && nx.kslot);
    gather_p_query<KS, false, true>(g, nx.sn, B, jp, mn, lane, nx.mu, nx.q64, nx.qn2, qf, ma.db64, nx.basis, nx.ufac,
                                    nx.qinfo, A, qsh[wv], pub ? xh[wv][0] : nullptr, xh[wv][1], h, o0, o1, o2, pf
#if IA_PROBE & 8
                                    , gprobe ? gst : nullptr
#endif
                                    );
    if (XO && nx.xp.W) xo_publish<KS>(nx.xp, mn, lane, xh[wv][0], xh[wv][1], o0, o1, o2);
    if (!XO && nx.kslot) sorted_publish<KS>(nx, mn, lane, xh[wv][0], xh[wv][1], o0, o1, o2);
  } else {
    gather_h_query_fused<KS>(g, nx.sn, B, mn, lane, nx.mu, nx.q64, nx.qn2, qf, h);
  }
#if IA_PROBE & 8
  __builtin_amdgcn_s_waitcnt(0);
  gs[3] = __builtin_amdgcn_s_memtime();
  if (gprobe && lane == 0)
    printf("GSTAMP bw=%d t=%d M=%d merge=%llu handoff_wait=%llu gather=%llu [feat+frag=%llu sums=%llu urow=%llu rec=%llu]\n",
           g.bw, sd.t, sd.M, gs[1] - gs[0], gs[2] - gs[1], gs[3] - gs[2], gst[1] - gst[0], gst[2] - gst[1], gst[3] - gst[2],
           gst[4] - gst[3]);
#endif
}
template <int RPL, bool PR, bool XO, class JS>
__global__ void __launch_bounds__(IA_PQ_WG) k_merge_gather(LevelGeo g, StepDesc sd, Imgs A, MergeArgs ma, JS jobs,
                                                         Imgs B, NextStep nx) {
  const unsigned long long t0 = ma.stamp ? ia_clock() : 0ull;  // option "stamps"
  merge_gather_body<RPL, PR, XO, JS>(g, sd, A, ma, jobs, B, nx);
  if (ma.stamp && (threadIdx.x & 63) == 0) ia_stamp_wg(ma.stamp, t0);
}

// multi-rank finish: global winner over the all-gathered per-rank winners, then coherence
template <int CH, class JS>
__global__ void __launch_bounds__(IA_WG) k_finish_level(LevelGeo g, StepDesc sd, Imgs A, const double *__restrict__ db64,
                                                         const double *__restrict__ q64,
                                                         const Winner *__restrict__ allwin, int world, int Mstride,
                                                         JS jobs) {
  const int m = __builtin_amdgcn_readfirstlane(blockIdx.x * (IA_WG / IA_WAVE) + (threadIdx.x >> 6));  // wave-uniform
  if (m >= sd.J * sd.M) return;
  double bd = DBL_MAX;
  int64_t bi = INT64_MAX;
  for (int k = 0; k < world; k++) {  // same order on every rank -> identical replicas
    const Winner w = allwin[(int64_t)k * Mstride + m];
    if (w.d < bd || (w.d == bd && w.idx < bi)) { bd = w.d; bi = w.idx; }
  }
  const QPix px = ia_qpix(sd, g.bw, m);
  const JobPtrs jp = jobs.get(px.job);
  const unsigned prev = jp.pstat ? jp.pstat[px.qi] : 0u;
  finish_pixel<CH>(g, A, db64, px.r, px.c, bi, q64 + (int64_t)m * Geo<CH>::D, jp.s, jp.im, jp.Bp, jp.weights, jp.kf,
                   jp.pstat, prev, jp.nn);
}

// Sharded level, peer-write exchange (option "exchange" = 1): the certified winner of this
// rank's shard (as k_merge_level<FUSED = false>) is written into every rank's exchange buffer;
// with FIN the wave then polls its own buffer for the W winners of its query, takes the global
// winner (smallest exact distance, then lowest row: the lexicographic minimum, independent of
// arrival order) and finishes the pixel (coherence, kappa, writeback) exactly as
// k_finish_level.  One launch per step replaces merge + all-gather + finish.  Emulated shards on
// one device (shard_emulate) publish with FIN = false for shards 0..W-2 and FIN = true for the
// last.  A wait beyond xa.timeout_ticks sets *err and finishes with the winners that arrived
// (the host reports IA_ECOMM): no wave spins forever.
template <int CH, bool FIN, class JS, int RPL>
__global__ void __launch_bounds__(IA_PQ_WG) k_merge_xchg(LevelGeo g, StepDesc sd, Imgs A, MergeArgs ma, XchgArgs xa, JS jobs) {
  const int m = __builtin_amdgcn_readfirstlane(blockIdx.x * IA_PQ_WPB + (threadIdx.x >> 6));  // wave-uniform
  if (m >= sd.J * sd.M) return;
  const int lane = threadIdx.x & 63;
  const QPix px = ia_qpix(sd, g.bw, m);
  const JobPtrs jp = jobs.get(px.job);
  const double *q = ma.q64 + (int64_t)m * Geo<CH>::D;
  unsigned stat = 0;
  const Winner wn = certified_winner<RPL>(ma, m, [&](int64_t row) { return exact_dist_level<CH>(ma.db64, row, q); }, &stat);
  if (lane < xa.W) {  // lane p publishes to rank p
    XSlot *sl = xa.peer[lane] + ia_xslot(xa.seq, xa.W, xa.rank, m);
    const unsigned row = wn.idx == INT64_MAX ? 0xffffffffu : (unsigned)wn.idx;
    __hip_atomic_store(reinterpret_cast<unsigned long long *>(&sl->d), (unsigned long long)__double_as_longlong(wn.d),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    ia_stores_done();  // the distance has reached the (uncached) slot before its (row, seq) word
    __hip_atomic_store(&sl->row_seq, (unsigned long long)row | ((unsigned long long)xa.seq << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if constexpr (!FIN) {
    if (lane == 0 && jp.pstat) jp.pstat[px.qi] = stat;
    return;
  } else {
    // the coherence pick does not depend on the NN winner: it runs while the peers' winners travel
    const CohPick ck = coherence_pick<CH>(g, ma.db64, px.r, px.c, q, jp.s, jp.im);
    double bd = DBL_MAX;
    int64_t bi = INT64_MAX;
    bool late = false;
    if (lane < xa.W) {  // lane p reads rank p's winner
      XSlot *sl = xa.local + ia_xslot(xa.seq, xa.W, lane, m);
      const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
      // after an earlier timeout of this context: no waiting (one lost peer costs one timeout)
      const long long lim = __hip_atomic_load(xa.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? -1 : xa.timeout_ticks;
      unsigned long long rs = __hip_atomic_load(&sl->row_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      while ((unsigned)(rs >> 32) != xa.seq) {
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > lim) {
          late = true;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
        rs = __hip_atomic_load(&sl->row_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (!late) {
        const unsigned long long db =
            __hip_atomic_load(reinterpret_cast<unsigned long long *>(&sl->d), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned row = (unsigned)rs;
        if (row < (unsigned)ma.NA) {  // 0xffffffff: the shard holds no row within the bound
          bd = __longlong_as_double((long long)db);
          bi = (int64_t)row;
        }
      }
    }
    if (__ballot(late) != 0ull && lane == 0) atomicOr(xa.err, 1u);
    wave_min_di(bd, bi);  // lexicographic (d, row) minimum: the same on every rank
    if (bi == INT64_MAX) {  // no shard reported a row (only after a timeout): keep every index in range
      bi = 0;
      if (lane == 0) atomicOr(xa.err, 2u);
    }
    finish_pick<CH>(g, A, ma.db64, px.r, px.c, bi, ck, q, jp.s, jp.im, jp.Bp, jp.weights, jp.kf, jp.pstat, stat, jp.nn);
  }
}

// per-level statistics: sum the per-pixel stats words.  Grid-stride loop over up to 256
// workgroups; each workgroup reduces in LDS and adds its five integer sums with one u64
// atomicAdd per counter (integer sums are order-free; counters are zeroed per level)
// option "stamps": launch i's first workgroup start and last workgroup end over its `stride`
// workgroup slots (unwritten slots are zero), in s_memrealtime ticks; one wave per launch
// span2 (optional): per launch the last workgroup start - the first, and the mean workgroup
// duration (ticks)
__global__ void __launch_bounds__(IA_WAVE) k_stamp_durations(const unsigned long long *__restrict__ stamps, int stride,
                                                            unsigned long long *__restrict__ span,
                                                            unsigned long long *__restrict__ span2) {
  const int i = blockIdx.x, lane = threadIdx.x;
  unsigned long long lo = ~0ull, hi = 0ull, smax = 0ull, dsum = 0ull, n = 0ull;
  for (int j = lane; j < stride; j += IA_WAVE) {
    const unsigned long long a = stamps[2 * ((int64_t)i * stride + j)], b = stamps[2 * ((int64_t)i * stride + j) + 1];
    if (a) {
      lo = a < lo ? a : lo;
      hi = b > hi ? b : hi;
      smax = a > smax ? a : smax;
      dsum += b > a ? b - a : 0ull;
      n++;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long l2 = __shfl_xor(lo, o, 64), h2 = __shfl_xor(hi, o, 64), m2 = __shfl_xor(smax, o, 64);
    lo = l2 < lo ? l2 : lo;
    hi = h2 > hi ? h2 : hi;
    smax = m2 > smax ? m2 : smax;
    dsum += __shfl_xor(dsum, o, 64);
    n += __shfl_xor(n, o, 64);
  }
  if (lane == 0) {
    const bool ok = hi >= lo && hi;
    span[2 * i] = ok ? lo : 0ull;
    span[2 * i + 1] = ok ? hi : 0ull;
    if (span2) {
      span2[2 * i] = ok ? smax - lo : 0ull;
      span2[2 * i + 1] = ok && n ? dsum / n : 0ull;
    }
  }
}
void ia_launch_stamp_durations(const unsigned long long *stamps, int n, int stride, unsigned long long *span, hipStream_t st,
                               unsigned long long *span2) {
  if (n > 0) hipLaunchKernelGGL(k_stamp_durations, dim3(n), dim3(IA_WAVE), 0, st, stamps, stride, span, span2);
}

__global__ void __launch_bounds__(IA_WG) k_reduce_stats(const unsigned *__restrict__ pstat, int64_t n,
                                                         unsigned long long *__restrict__ counters) {
  unsigned long long rr = 0, fb = 0, cw = 0, bv = 0, ka = 0;
  for (int64_t i = (int64_t)blockIdx.x * IA_WG + threadIdx.x; i < n; i += (int64_t)gridDim.x * IA_WG) {
    const unsigned v = pstat[i];
    rr += v & 0xffff;
    fb += (v >> 16) & 0x1fff;
    ka += (v >> 29) & 1;
    cw += (v >> 30) & 1;
    bv += v >> 31;
  }
  __shared__ unsigned long long red[5][IA_WG];
  red[0][threadIdx.x] = rr;
  red[1][threadIdx.x] = fb;
  red[2][threadIdx.x] = cw;
  red[3][threadIdx.x] = bv;
  red[4][threadIdx.x] = ka;
  __syncthreads();
  for (int o = IA_WG / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
      for (int k = 0; k < 5; k++) red[k][threadIdx.x] += red[k][threadIdx.x + o];
    __syncthreads();
  }
  // integer sums: order-free, so one global atomic per counter and workgroup (counters are
  // zeroed at the start of the level)
  if (threadIdx.x < 5) atomicAdd(&counters[threadIdx.x], red[threadIdx.x][0]);
}

// ------------------------------------------------------------------------------------------
// dense (FLANN-compatible index) variants: rows given as n x d fp64
// ------------------------------------------------------------------------------------------
template <int KH>
__global__ void __launch_bounds__(IA_WG) k_dense_db_build(const double *__restrict__ pts, int64_t n, int d, int n_tiles,
                                                           const double *__restrict__ mu, float4 *__restrict__ db,
                                                           unsigned *__restrict__ Rbits) {
  constexpr int KP = KH / 4;
  const int64_t pos = (int64_t)blockIdx.x * IA_WG + threadIdx.x;
  if (pos >= (int64_t)n_tiles * IA_TILE) return;
  const int64_t row = ia_pos_row(pos, n_tiles);
  const bool real = row < n;
  const int64_t tile = pos / IA_TILE;
  const int j = (int)(pos % IA_TILE);
  double norm = 0.;
  for (int h = 0; h < 2; h++) {
    for (int p = 0; p < KP; p++) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int f = h * KH + 4 * p + e;
        if (f < d) {
          double a = real ? pts[row * d + f] - mu[f] : 0.;
          norm += a * a;
          v[e] = (float)a;
        } else if (f == d) {
          v[e] = real ? (float)norm : IA_PAD_NORM;
        } else {
          v[e] = 0.f;
        }
      }
      db[(tile * KP + p) * IA_WAVE + h * IA_TILE + j] = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
  if (real) atomicMax(Rbits, __float_as_uint((float)(sqrt(norm) * (1.0 + 1e-6))));
}

template <int KH>
__global__ void __launch_bounds__(IA_WG) k_dense_query(const double *__restrict__ q, int64_t nq, int d, int Mpad,
                                                        const double *__restrict__ mu, double *__restrict__ qn2,
                                                        float *__restrict__ qf) {
  constexpr int KP = KH / 4;
  const int lane = threadIdx.x & 63;
  const int m = __builtin_amdgcn_readfirstlane(blockIdx.x * (IA_WG / IA_WAVE) + (threadIdx.x >> 6));  // wave-uniform
  if (m >= Mpad) return;
  double ss = 0.;
  for (int f = lane; f < 2 * KH; f += IA_WAVE) {
    float v = 0.f;
    if (m < nq && f < d) {
      const double qc = q[(int64_t)m * d + f] - mu[f];
      ss += qc * qc;
      v = -2.f * (float)qc;
    } else if (m < nq && f == d) {
      v = 1.f;
    }
    const int qt = m / IA_TILE, j = m % IA_TILE, h = f / KH, s = f % KH;
    qf[(((int64_t)qt * KP + s / 4) * IA_WAVE + h * IA_TILE + j) * 4 + (s % 4)] = v;
  }
  ss = wave_sum_d(ss);
  if (lane == 0 && m < nq) qn2[m] = ss;
}

__global__ void __launch_bounds__(IA_WG) k_merge_dense(MergeArgs ma, const double *__restrict__ pts, int d, const double *__restrict__ q,
                                                        int64_t nq, int64_t *__restrict__ idx_out, double *__restrict__ dist_out) {
  const int m = __builtin_amdgcn_readfirstlane(blockIdx.x * (IA_WG / IA_WAVE) + (threadIdx.x >> 6));  // wave-uniform
  if (m >= nq) return;
  const double *qm = q + (int64_t)m * d;
  unsigned stat;
  const Winner wn = certified_winner(ma, m, [&](int64_t row) {
    const double *a = pts + row * d;
    return pw_sum_rt([&](int f) {
      const double x = a[f] - qm[f];
      return x * x;
    }, d);
  }, &stat);
  if ((threadIdx.x & 63) == 0) {
    idx_out[m] = wn.idx;
    dist_out[m] = wn.d;
  }
}

// best_coherence_match (algorithms.py:92-130) for a batch of B' pixels against an index's rows,
// one wave per pixel.  Lane j < (pad+1)(2 pad+1) is the window cell (row - pad + j / (2 pad+1),
// col - pad + j % (2 pad+1)), i.e. product(rows, cols) order (:101-104); a cell is a candidate
// when it is inside the level, raster-earlier (:107) and its shifted source s[r] + (q - r) lies
// inside A (:116).  Distance = sqrt of numpy's pairwise sum of squares (norm(..., axis=1),
// :126), first argmin.  err bit 0: an s index beyond n_s; bit 1: a DB row beyond the index.
__global__ void __launch_bounds__(IA_WG) k_coherence_batch(const double *__restrict__ pts, int64_t n, int d,
                                                            const double *__restrict__ q, int64_t nq,
                                                            const int32_t *__restrict__ px, const int32_t *__restrict__ s,
                                                            const int32_t *__restrict__ im, int64_t n_s, int a_h, int a_w,
                                                            int bp_w, int pad, int32_t *__restrict__ p_out,
                                                            int32_t *__restrict__ img_out, int32_t *__restrict__ r_out,
                                                            unsigned *__restrict__ err) {
  const int m = __builtin_amdgcn_readfirstlane(blockIdx.x * (IA_WG / IA_WAVE) + (threadIdx.x >> 6));  // wave-uniform
  const int lane = threadIdx.x & 63;
  if (m >= nq) return;
  const int row = px[2 * m], col = px[2 * m + 1], wd = 2 * pad + 1;
  const int rr = row - pad + lane / wd, rc = col - pad + lane % wd;
  const int64_t here = (int64_t)row * bp_w + col, ri = (int64_t)rr * bp_w + rc;
  bool ok = lane < (pad + 1) * wd && rr >= 0 && rc >= 0 && rc < bp_w && ri < here;
  int pr0 = 0, pr1 = 0, img = 0;
  int64_t dbrow = 0;
  unsigned e = 0;
  if (ok && ri >= n_s) {
    e |= 1u;
    ok = false;
  }
  if (ok) {
    pr0 = s[2 * ri] + row - rr;
    pr1 = s[2 * ri + 1] + col - rc;
    img = im[ri];
    ok = pr0 >= 0 && pr0 < a_h && pr1 >= 0 && pr1 < a_w;
    dbrow = ((int64_t)img * a_h + pr0) * a_w + pr1;
    if (ok && (dbrow < 0 || dbrow >= n)) {
      e |= 2u;
      ok = false;
    }
  }
  double dist = INFINITY;
  int64_t key = ok ? lane : 64;
  if (ok) {
    const double *a = pts + dbrow * d, *qm = q + (int64_t)m * d;
    dist = cr_sqrt(pw_sum_rt([&](int f) {
      const double x = a[f] - qm[f];
      return x * x;
    }, d));
  }
  if (e) atomicOr(err, e);
  wave_min_di(dist, key);  // first argmin (lowest window cell) among the candidates
  if (key >= 64) {
    if (lane == 0) {
      p_out[2 * m] = -1;
      p_out[2 * m + 1] = -1;
      img_out[m] = 0;
      r_out[2 * m] = 0;
      r_out[2 * m + 1] = 0;
    }
    return;
  }
  if (lane == (int)key) {  // s[r*] + q - r*, im[r*], r*
    p_out[2 * m] = pr0;
    p_out[2 * m + 1] = pr1;
    img_out[m] = img;
    r_out[2 * m] = rr;
    r_out[2 * m + 1] = rc;
  }
}

// ------------------------------------------------------------------------------------------
// host-side launchers (called from ia_capi.cpp)
// ------------------------------------------------------------------------------------------
#include "ia_launch.h"

static inline unsigned cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }
static inline Imgs job0_imgs(Imgs B, const JobSet &jobs) {  // a single job's images in the Imgs argument
  B.p0 = jobs.j0.Bc;
  B.p1 = jobs.j0.B;
  B.p2 = jobs.j0.Bpc;
  B.p3 = jobs.j0.Bp;
  return B;
}

template <int CH>
static void launch_means_t(const Imgs &A, int n_ap, double *mu, hipStream_t st) {
  // partial sums live behind the 4 CH means in the same buffer (ia_capi.cpp sizes it)
  double *parts = mu + 16;
  hipLaunchKernelGGL(k_part_means<CH>, dim3(IA_MEAN_CHUNKS, 4 * CH), dim3(IA_WG), 0, st, A, n_ap, parts);
  hipLaunchKernelGGL(k_part_means_fold<CH>, dim3(1), dim3(IA_WG), 0, st, A, n_ap, (const double *)parts, mu);
}
void ia_launch_means(int ch, const Imgs &A, int n_ap, double *mu, hipStream_t st) {
  if (ch == 1) launch_means_t<1>(A, n_ap, mu, st);
  else if (ch == 2) launch_means_t<2>(A, n_ap, mu, st);
  else launch_means_t<3>(A, n_ap, mu, st);
}

template <int CH>
static void launch_db_t(const LevelGeo &g, const Imgs &A, const double *mu, float4 *db, unsigned *Rbits, hipStream_t st) {
  const int64_t rows = (int64_t)(g.tile1 - g.tile0) * IA_TILE;
  hipLaunchKernelGGL(k_db_build<CH>, dim3(cdiv(rows, IA_WG)), dim3(IA_WG), 0, st, g, A, mu, db, Rbits);
}
void ia_launch_db_build(const LevelGeo &g, const Imgs &A, const double *mu, float4 *db, unsigned *Rbits, hipStream_t st) {
  if (g.ch == 1) launch_db_t<1>(g, A, mu, db, Rbits, st);
  else if (g.ch == 2) launch_db_t<2>(g, A, mu, db, Rbits, st);
  else launch_db_t<3>(g, A, mu, db, Rbits, st);
}

template <int CH>
static void launch_gather_t(const LevelGeo &g, const StepDesc &sd, const Imgs &B, const JobSet &jobs, const double *mu,
                            double *q64, double *qn2, float *qf, hipStream_t st) {
  const dim3 grid(cdiv(sd.Mpad, IA_WG / IA_WAVE));
  if (jobs.J == 1)
    hipLaunchKernelGGL((k_gather_query<CH, JobArg1>), grid, dim3(IA_WG), 0, st, g, sd, job0_imgs(B, jobs), JobArg1{jobs.j0}, mu,
                       q64, qn2, qf);
  else
    hipLaunchKernelGGL((k_gather_query<CH, JobArgN>), grid, dim3(IA_WG), 0, st, g, sd, B, JobArgN{jobs.rest}, mu, q64, qn2, qf);
}
void ia_launch_gather(const LevelGeo &g, const StepDesc &sd, const Imgs &B, const JobSet &jobs, const double *mu, double *q64,
                      double *qn2, float *qf, hipStream_t st) {
  if (g.ch == 1) launch_gather_t<1>(g, sd, B, jobs, mu, q64, qn2, qf, st);
  else if (g.ch == 2) launch_gather_t<2>(g, sd, B, jobs, mu, q64, qn2, qf, st);
  else launch_gather_t<3>(g, sd, B, jobs, mu, q64, qn2, qf, st);
}

// K3 dispatch table: QT query tiles per launch (1..QTMAX(KH))
typedef void (*k3_fn)(const float4 *, const float4 *, int, int, int, int, int, int, int, float4 *, float *);
template <int KH, int... QTs>
struct K3Table {
  static k3_fn get(int qt) {
    static const k3_fn tab[] = {k3_dist<KH, QTs>...};
    return tab[qt - 1];
  }
};
int ia_k3_qtmax(int KH) { return KH == 28 ? 11 : KH == 56 ? 5 : 3; }

// Allow a kernel the architecture's whole LDS as dynamic shared memory (gfx950: 160 KiB per CU;
// the default cap is 64 KiB), once per kernel.  Several host threads launch through one libia
// (one context each: DeviceSweep, bench --streams), so the set is guarded; the attribute is the
// arch maximum rather than the launch's size, so no thread can lower it under another's launch.
static void allow_full_lds(const void *fn) {
  static std::mutex mu;
  static std::unordered_set<const void *> done;
  std::lock_guard<std::mutex> lk(mu);
  if (!done.insert(fn).second) return;
  hipFuncAttributes fa;  // dynamic + static shared memory must fit the CU's 160 KiB
  const int stat = hipFuncGetAttributes(&fa, fn) == hipSuccess ? (int)fa.sharedSizeBytes : 1024;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - stat);
}

void ia_launch_k3(int KH, int qt, const float4 *db, const float4 *qf, int n_tiles, int tpw, int qt0, int M, int nwg,
                  int row0, int NT, float4 *rec, float *recT, hipStream_t st) {
  k3_fn fn;
  if (KH == 28) fn = K3Table<28, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11>::get(qt);
  else if (KH == 56) fn = K3Table<56, 1, 2, 3, 4, 5>::get(qt);
  else fn = K3Table<84, 1, 2, 3>::get(qt);
  const size_t lds = (size_t)qt * (KH / 4) * IA_WAVE * sizeof(float4);
  allow_full_lds((const void *)fn);
  hipLaunchKernelGGL(fn, dim3(nwg), dim3(IA_WG), lds, st, db, qf, n_tiles, tpw, qt0, M, nwg, row0, NT, rec, recT);
}

template <int CH, bool FUSED, bool IMG>
static void launch_merge_j(const LevelGeo &g, const StepDesc &sd, const Imgs &A, const MergeArgs &ma, Winner *win,
                           const JobSet &jobs, hipStream_t st) {
  const dim3 grid(cdiv(sd.J * sd.M, IA_PQ_WPB));
  // the fused merge with 4 records per lane when the scan ran <= 256 workgroups (every
  // split-f16 scan): half the record loads and candidate tests of the 8-per-lane form
  const bool r4 = FUSED && ma.nwg <= 4 * IA_WAVE && !IA_K4_RPL8;
  if (jobs.J == 1) {
    if (r4)
      hipLaunchKernelGGL((k_merge_level<CH, FUSED, IMG, JobArg1, 4>), grid, dim3(IA_PQ_WG), 0, st, g, sd, A, ma, win, JobArg1{jobs.j0});
    else
      hipLaunchKernelGGL((k_merge_level<CH, FUSED, IMG, JobArg1>), grid, dim3(IA_PQ_WG), 0, st, g, sd, A, ma, win, JobArg1{jobs.j0});
  } else {
    if (r4)
      hipLaunchKernelGGL((k_merge_level<CH, FUSED, IMG, JobArgN, 4>), grid, dim3(IA_PQ_WG), 0, st, g, sd, A, ma, win,
                         JobArgN{jobs.rest});
    else
      hipLaunchKernelGGL((k_merge_level<CH, FUSED, IMG, JobArgN>), grid, dim3(IA_PQ_WG), 0, st, g, sd, A, ma, win,
                         JobArgN{jobs.rest});
  }
}
void ia_launch_merge_gather(const LevelGeo &g, const StepDesc &sd, const Imgs &A, const MergeArgs &ma, const JobSet &jobs,
                            const Imgs &B, const NextStep &nx, bool pruned, hipStream_t st) {
  // waves: the step's merges, each job's entering row, the next step's pad queries (+ the waiter)
  const int nw = sd.J * sd.M + sd.J + (nx.sn.Mpad - sd.J * nx.sn.M) + (nx.wait_n > 0 ? 1 : 0);
  const dim3 grid(cdiv(nw, IA_PQ_WPB));
  const bool xo = nx.xp.W > 0 || nx.wait_n > 0;
  if (jobs.J == 1 && pruned && xo)
    hipLaunchKernelGGL((k_merge_gather<4, true, true, JobArg1>), grid, dim3(IA_PQ_WG), 0, st, g, sd, A, ma, JobArg1{jobs.j0},
                       job0_imgs(B, jobs), nx);
  else if (jobs.J == 1 && pruned)
    hipLaunchKernelGGL((k_merge_gather<4, true, false, JobArg1>), grid, dim3(IA_PQ_WG), 0, st, g, sd, A, ma, JobArg1{jobs.j0},
                       job0_imgs(B, jobs), nx);
  else if (jobs.J == 1)
    hipLaunchKernelGGL((k_merge_gather<4, false, false, JobArg1>), grid, dim3(IA_PQ_WG), 0, st, g, sd, A, ma, JobArg1{jobs.j0},
                       job0_imgs(B, jobs), nx);
  else if (pruned)
    hipLaunchKernelGGL((k_merge_gather<4, true, false, JobArgN>), grid, dim3(IA_PQ_WG), 0, st, g, sd, A, ma, JobArgN{jobs.rest},
                       B, nx);
  else
    hipLaunchKernelGGL((k_merge_gather<4, false, false, JobArgN>), grid, dim3(IA_PQ_WG), 0, st, g, sd, A, ma, JobArgN{jobs.rest},
                       B, nx);
}
// the chained-wave budget's inputs (ia_capi.cpp, ia_chain_budget): over every k_merge_gather
// instance the library launches, the most VGPRs per lane and the fewest workgroups per CU the
// occupancy API admits, from the compiled kernels themselves
void ia_merge_gather_occupancy(int *vgprs, int *blocks_per_cu, int *wg_threads) {
  const void *fns[] = {(const void *)k_merge_gather<4, true, true, JobArg1>, (const void *)k_merge_gather<4, true, false, JobArg1>,
                       (const void *)k_merge_gather<4, false, false, JobArg1>, (const void *)k_merge_gather<4, true, false, JobArgN>,
                       (const void *)k_merge_gather<4, false, false, JobArgN>};
  int vmax = 0, bmin = 1 << 30;
  for (const void *fn : fns) {
    hipFuncAttributes fa;
    int nb = 0;
    if (hipFuncGetAttributes(&fa, fn) != hipSuccess || hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, IA_PQ_WG, 0) != hipSuccess) {
      bmin = 0;
      continue;
    }
    vmax = std::max(vmax, (int)fa.numRegs);
    bmin = std::min(bmin, nb);
  }
  *vgprs = vmax;
  *blocks_per_cu = bmin;
  *wg_threads = IA_PQ_WG;
}
template <int CH>
static void launch_merge_t(const LevelGeo &g, const StepDesc &sd, const Imgs &A, const MergeArgs &ma, Winner *win,
                           const JobSet &jobs, bool fused, hipStream_t st) {
  if (fused) launch_merge_j<CH, true, false>(g, sd, A, ma, win, jobs, st);
  else launch_merge_j<CH, false, false>(g, sd, A, ma, win, jobs, st);
}
void ia_launch_merge(const LevelGeo &g, const StepDesc &sd, const Imgs &A, const MergeArgs &ma, Winner *win,
                     const JobSet &jobs, bool fused, hipStream_t st) {
  if (g.ch == 1) launch_merge_t<1>(g, sd, A, ma, win, jobs, fused, st);
  else if (g.ch == 2) launch_merge_t<2>(g, sd, A, ma, win, jobs, fused, st);
  else launch_merge_t<3>(g, sd, A, ma, win, jobs, fused, st);
}

template <int CH>
static void launch_finish_t(const LevelGeo &g, const StepDesc &sd, const Imgs &A, const double *db64, const double *q64,
                            const Winner *allwin, int world, int Mstride, const JobSet &jobs, hipStream_t st) {
  const dim3 grid(cdiv(sd.J * sd.M, IA_WG / IA_WAVE));
  if (jobs.J == 1)
    hipLaunchKernelGGL((k_finish_level<CH, JobArg1>), grid, dim3(IA_WG), 0, st, g, sd, A, db64, q64, allwin, world, Mstride,
                       JobArg1{jobs.j0});
  else
    hipLaunchKernelGGL((k_finish_level<CH, JobArgN>), grid, dim3(IA_WG), 0, st, g, sd, A, db64, q64, allwin, world, Mstride,
                       JobArgN{jobs.rest});
}
void ia_launch_finish(const LevelGeo &g, const StepDesc &sd, const Imgs &A, const double *db64, const double *q64,
                      const Winner *allwin, int world, int Mstride, const JobSet &jobs, hipStream_t st) {
  if (g.ch == 1) launch_finish_t<1>(g, sd, A, db64, q64, allwin, world, Mstride, jobs, st);
  else if (g.ch == 2) launch_finish_t<2>(g, sd, A, db64, q64, allwin, world, Mstride, jobs, st);
  else launch_finish_t<3>(g, sd, A, db64, q64, allwin, world, Mstride, jobs, st);
}

template <int CH, bool FIN, int RPL, class JS>
static void launch_xchg_j(const LevelGeo &g, const StepDesc &sd, const Imgs &A, const MergeArgs &ma, const XchgArgs &xa,
                          const JS &js, hipStream_t st) {
  hipLaunchKernelGGL((k_merge_xchg<CH, FIN, JS, RPL>), dim3(cdiv(sd.J * sd.M, IA_PQ_WPB)), dim3(IA_PQ_WG), 0, st, g, sd, A, ma,
                     xa, js);
}
template <int CH>
static void launch_xchg_t(const LevelGeo &g, const StepDesc &sd, const Imgs &A, const MergeArgs &ma, const XchgArgs &xa,
                          const JobSet &jobs, bool fin, hipStream_t st) {
  // 4 records per lane when the shard's scan ran <= 256 workgroups (every split-f16 scan)
  const bool r4 = ma.nwg <= 4 * IA_WAVE;
  if (jobs.J == 1) {
    if (fin && r4) launch_xchg_j<CH, true, 4>(g, sd, A, ma, xa, JobArg1{jobs.j0}, st);
    else if (fin) launch_xchg_j<CH, true, 8>(g, sd, A, ma, xa, JobArg1{jobs.j0}, st);
    else if (r4) launch_xchg_j<CH, false, 4>(g, sd, A, ma, xa, JobArg1{jobs.j0}, st);
    else launch_xchg_j<CH, false, 8>(g, sd, A, ma, xa, JobArg1{jobs.j0}, st);
  } else {  // several jobs per sharded level: every rank holds every job's replica
    if (fin && r4) launch_xchg_j<CH, true, 4>(g, sd, A, ma, xa, JobArgN{jobs.rest}, st);
    else if (fin) launch_xchg_j<CH, true, 8>(g, sd, A, ma, xa, JobArgN{jobs.rest}, st);
    else if (r4) launch_xchg_j<CH, false, 4>(g, sd, A, ma, xa, JobArgN{jobs.rest}, st);
    else launch_xchg_j<CH, false, 8>(g, sd, A, ma, xa, JobArgN{jobs.rest}, st);
  }
}
void ia_launch_merge_xchg(const LevelGeo &g, const StepDesc &sd, const Imgs &A, const MergeArgs &ma, const XchgArgs &xa,
                          const JobSet &jobs, bool fin, hipStream_t st) {
  if (g.ch == 1) launch_xchg_t<1>(g, sd, A, ma, xa, jobs, fin, st);
  else if (g.ch == 2) launch_xchg_t<2>(g, sd, A, ma, xa, jobs, fin, st);
  else launch_xchg_t<3>(g, sd, A, ma, xa, jobs, fin, st);
}

template <int CH>
static void launch_db64_t(const LevelGeo &g, const Imgs &A, double *db64, hipStream_t st) {
  hipLaunchKernelGGL(k_db64_build<CH>, dim3(cdiv(g.NA, IA_WAVE)), dim3(IA_WAVE), 0, st, g, A, db64);
}
void ia_launch_db64_build(const LevelGeo &g, const Imgs &A, double *db64, hipStream_t st) {
  if (g.ch == 1) launch_db64_t<1>(g, A, db64, st);
  else if (g.ch == 2) launch_db64_t<2>(g, A, db64, st);
  else launch_db64_t<3>(g, A, db64, st);
}
int ia_db64_stride(int ch) { return ch == 1 ? Geo<1>::DS : ch == 2 ? Geo<2>::DS : Geo<3>::DS; }

void ia_launch_reduce_stats(const unsigned *pstat, int64_t n, unsigned long long *counters, hipStream_t st) {
  const int64_t nwg = std::min<int64_t>(256, std::max<int64_t>(1, cdiv(n, (int64_t)IA_WG * 16)));
  hipLaunchKernelGGL(k_reduce_stats, dim3((unsigned)nwg), dim3(IA_WG), 0, st, pstat, n, counters);
}

void ia_launch_dense_db(int KH, const double *pts, int64_t n, int d, int n_tiles, const double *mu, float4 *db,
                        unsigned *Rbits, hipStream_t st) {
  dim3 grid(cdiv((int64_t)n_tiles * IA_TILE, IA_WG));
  if (KH == 28) hipLaunchKernelGGL(k_dense_db_build<28>, grid, dim3(IA_WG), 0, st, pts, n, d, n_tiles, mu, db, Rbits);
  else if (KH == 56) hipLaunchKernelGGL(k_dense_db_build<56>, grid, dim3(IA_WG), 0, st, pts, n, d, n_tiles, mu, db, Rbits);
  else hipLaunchKernelGGL(k_dense_db_build<84>, grid, dim3(IA_WG), 0, st, pts, n, d, n_tiles, mu, db, Rbits);
}
void ia_launch_dense_query(int KH, const double *q, int64_t nq, int d, int Mpad, const double *mu, double *qn2, float *qf,
                           hipStream_t st) {
  dim3 grid(cdiv(Mpad, IA_WG / IA_WAVE));
  if (KH == 28) hipLaunchKernelGGL(k_dense_query<28>, grid, dim3(IA_WG), 0, st, q, nq, d, Mpad, mu, qn2, qf);
  else if (KH == 56) hipLaunchKernelGGL(k_dense_query<56>, grid, dim3(IA_WG), 0, st, q, nq, d, Mpad, mu, qn2, qf);
  else hipLaunchKernelGGL(k_dense_query<84>, grid, dim3(IA_WG), 0, st, q, nq, d, Mpad, mu, qn2, qf);
}
void ia_launch_merge_dense(const MergeArgs &ma, const double *pts, int d, const double *q, int64_t nq, int64_t *idx,
                           double *dist, hipStream_t st) {
  hipLaunchKernelGGL(k_merge_dense, dim3(cdiv(nq, IA_WG / IA_WAVE)), dim3(IA_WG), 0, st, ma, pts, d, q, nq, idx, dist);
}
void ia_launch_coherence_batch(const double *pts, int64_t n, int d, const double *q, int64_t nq, const int32_t *px,
                               const int32_t *s, const int32_t *im, int64_t n_s, int a_h, int a_w, int bp_w, int pad,
                               int32_t *p_out, int32_t *img_out, int32_t *r_out, unsigned *err, hipStream_t st) {
  hipLaunchKernelGGL(k_coherence_batch, dim3(cdiv(nq, IA_WG / IA_WAVE)), dim3(IA_WG), 0, st, pts, n, d, q, nq, px, s, im, n_s,
                     a_h, a_w, bp_w, pad, p_out, img_out, r_out, err);
}

// ---- split-f16 matcher launchers -----------------------------------------------------------
double ia_k3h_tile_bytes(int KS) { return KS == 4 ? 16.0 * TileFmt<4>::STRIDE : KS == 7 ? 16.0 * TileFmt<7>::STRIDE : 0.; }
int ia_ks_for(int ch) { return ch == 1 ? 4 : ch == 2 ? 7 : 0; }  // 3 channels: fp32 matcher
int ia_k3h_qtmax(int KS) { return KS == 4 ? 11 : 8; }
// waves per workgroup of the K3h instance selected by (KS, qt, variant) (ia_k3h.hip getters)
static int k3h_waves(int KS, int qt, int variant) {
  return IA_WGH / IA_WAVE;
}
static size_t k3h_lds(int KS, int qt, int nw) {
  const size_t q = (size_t)qt * 2 * KS * IA_WAVE * 16, m = (size_t)nw * qt * IA_TILE * sizeof(Top2);
  return q > m ? q : m;
}
size_t ia_k3h_lds(int KS, int qt) {
  const size_t q = (size_t)qt * 2 * KS * IA_WAVE * 16, m = (size_t)(IA_WGH / IA_WAVE) * qt * IA_TILE * sizeof(Top2);
  return q > m ? q : m;
}

// microbenchmark operands: pseudo-random f16 values in [-0.5, 0.5) (hash of the index)
__global__ void __launch_bounds__(IA_WG) k_fill_random_f16(_Float16 *__restrict__ p, int64_t n, unsigned seed) {
  for (int64_t i = (int64_t)blockIdx.x * IA_WG + threadIdx.x; i < n; i += (int64_t)gridDim.x * IA_WG) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    p[i] = (_Float16)((float)(h & 0xffff) * (1.f / 65536.f) - 0.5f);
  }
}
void ia_launch_fill_random_f16(void *p, int64_t n, unsigned seed, hipStream_t st) {
  hipLaunchKernelGGL(k_fill_random_f16, dim3(1024), dim3(IA_WG), 0, st, (_Float16 *)p, n, seed);
}

void ia_launch_absmax(const double *const *p, const int64_t *n, unsigned *out, hipStream_t st) {
  AbsArrays arr;
  for (int k = 0; k < 8; k++) {
    arr.p[k] = p[k];
    arr.n[k] = p[k] ? n[k] : 0;
  }
  hipLaunchKernelGGL(k_absmax, dim3(512), dim3(IA_WG), 0, st, arr, out);
}

template <int CH, int KS>
static void launch_db_h_t(const LevelGeo &g, const Imgs &A, const double *db64, const double *mu, void *db, unsigned *Rbits,
                          hipStream_t st) {
  (void)A;
  const int64_t tiles = (int64_t)g.tile1 - g.tile0;  // one wave per tile, <= 4 tiles per wave
  const int64_t nwg = std::max<int64_t>(1, std::min<int64_t>(cdiv(tiles, IA_WG / IA_WAVE), 2048));
  hipLaunchKernelGGL((k_db_build_h<CH, KS>), dim3((unsigned)nwg), dim3(IA_WG), 0, st, g, db64, mu, (h16x8 *)db, Rbits);
}
void ia_launch_db_build_h(const LevelGeo &g, const Imgs &A, const double *db64, const double *mu, void *db, unsigned *Rbits,
                          hipStream_t st) {
  if (g.ch == 1) launch_db_h_t<1, 4>(g, A, db64, mu, db, Rbits, st);
  else launch_db_h_t<2, 7>(g, A, db64, mu, db, Rbits, st);
}

template <int CH, int KS>
static void launch_gather_h_t(const LevelGeo &g, const StepDesc &sd, const Imgs &B, const JobSet &jobs, const double *mu,
                              double *q64, double *qn2, void *qf, hipStream_t st) {
  const dim3 grid(cdiv(sd.Mpad, IA_PQ_WPB));
  if (jobs.J == 1)
    hipLaunchKernelGGL((k_gather_query_h<CH, KS, JobArg1>), grid, dim3(IA_PQ_WG), 0, st, g, sd, job0_imgs(B, jobs), JobArg1{jobs.j0},
                       mu, q64, qn2, (_Float16 *)qf);
  else
    hipLaunchKernelGGL((k_gather_query_h<CH, KS, JobArgN>), grid, dim3(IA_PQ_WG), 0, st, g, sd, B, JobArgN{jobs.rest}, mu, q64,
                       qn2, (_Float16 *)qf);
}
void ia_launch_gather_h(const LevelGeo &g, const StepDesc &sd, const Imgs &B, const JobSet &jobs, const double *mu,
                        double *q64, double *qn2, void *qf, hipStream_t st) {
  if (g.ch == 1) launch_gather_h_t<1, 4>(g, sd, B, jobs, mu, q64, qn2, qf, st);
  else launch_gather_h_t<2, 7>(g, sd, B, jobs, mu, q64, qn2, qf, st);
}

template <bool IMG>
static void launch_gather_p_t(const LevelGeo &g, const StepDesc &sd, const Imgs &B, const JobSet &jobs, const double *mu,
                              double *q64, double *qn2, void *qf, const double *db64, const double *basis, double ufac,
                              float4 *qinfo, const Imgs &A, const XOPub &xp, hipStream_t st) {
  const dim3 grid(cdiv(sd.Mpad, IA_PQ_WPB));
  if (jobs.J == 1)
    hipLaunchKernelGGL((k_gather_query_p<4, IMG, JobArg1>), grid, dim3(IA_PQ_WG), 0, st, g, sd, job0_imgs(B, jobs), JobArg1{jobs.j0},
                       mu, q64, qn2, (_Float16 *)qf, db64, basis, ufac, qinfo, A, xp);
  else
    hipLaunchKernelGGL((k_gather_query_p<4, IMG, JobArgN>), grid, dim3(IA_PQ_WG), 0, st, g, sd, B, JobArgN{jobs.rest}, mu, q64,
                       qn2, (_Float16 *)qf, db64, basis, ufac, qinfo, A, xp);
}
void ia_launch_gather_p(const LevelGeo &g, const StepDesc &sd, const Imgs &B, const JobSet &jobs, const double *mu,
                        double *q64, double *qn2, void *qf, const double *db64, const double *basis, double ufac,
                        float4 *qinfo, const Imgs &A, int img_rows, hipStream_t st, const XOPub *xp) {
  const XOPub x = xp ? *xp : XOPub{};
  (void)img_rows;
  launch_gather_p_t<false>(g, sd, B, jobs, mu, q64, qn2, qf, db64, basis, ufac, qinfo, A, x, st);
}


// split-f16 distance kernels live in ia_k3h.hip, compiled once per (KS, QT) instance
#define IA_K3H_DECL(ks, qt) k3h_fn ia_k3h_get_##ks##_##qt(int variant);
IA_K3H_DECL(4, 1) IA_K3H_DECL(4, 2) IA_K3H_DECL(4, 3) IA_K3H_DECL(4, 4) IA_K3H_DECL(4, 5) IA_K3H_DECL(4, 6)
IA_K3H_DECL(4, 7) IA_K3H_DECL(4, 8) IA_K3H_DECL(4, 9) IA_K3H_DECL(4, 10) IA_K3H_DECL(4, 11)
IA_K3H_DECL(7, 1) IA_K3H_DECL(7, 2) IA_K3H_DECL(7, 3) IA_K3H_DECL(7, 4) IA_K3H_DECL(7, 5) IA_K3H_DECL(7, 6)
IA_K3H_DECL(7, 7) IA_K3H_DECL(7, 8)
static k3h_fn k3h_get(int KS, int qt, int variant) {
  typedef k3h_fn (*getter)(int);
  static const getter g4[] = {ia_k3h_get_4_1, ia_k3h_get_4_2, ia_k3h_get_4_3, ia_k3h_get_4_4,  ia_k3h_get_4_5, ia_k3h_get_4_6,
                              ia_k3h_get_4_7, ia_k3h_get_4_8, ia_k3h_get_4_9, ia_k3h_get_4_10, ia_k3h_get_4_11};
  static const getter g7[] = {ia_k3h_get_7_1, ia_k3h_get_7_2, ia_k3h_get_7_3, ia_k3h_get_7_4,
                              ia_k3h_get_7_5, ia_k3h_get_7_6, ia_k3h_get_7_7, ia_k3h_get_7_8};
  return KS == 4 ? g4[qt - 1](variant) : g7[qt - 1](variant);
}
void ia_launch_k3h(int KS, int qt, const void *db, const void *qf, int n_tiles, int tpw, int qt0, int M, int nwg, int row0,
                   int NT, float4 *rec, float *recT, int variant, hipStream_t st) {
  const k3h_fn fn = k3h_get(KS, qt, variant);
  const int nw = k3h_waves(KS, qt, variant);
  const size_t lds = k3h_lds(KS, qt, nw);
  allow_full_lds((const void *)fn);
  hipLaunchKernelGGL(fn, dim3(nwg), dim3(nw * IA_WAVE), lds, st, (const h16x8 *)db, (const h16x8 *)qf, n_tiles, tpw, qt0, M, nwg,
                     row0, NT, rec, recT);
}

// pruned split-f16 distance kernels (ia_k3h.hip k3h_prune, 1 channel)
#define IA_K3P_DECL(qt) k3p_fn ia_k3p_get_4_##qt(int);
IA_K3P_DECL(1) IA_K3P_DECL(2) IA_K3P_DECL(3) IA_K3P_DECL(4) IA_K3P_DECL(5) IA_K3P_DECL(6) IA_K3P_DECL(7) IA_K3P_DECL(8)
IA_K3P_DECL(9) IA_K3P_DECL(10) IA_K3P_DECL(11)
size_t ia_k3p_lds(int qt, int Mpad) {
  const size_t NQ = (size_t)qt * IA_TILE;
  const size_t qfrag = (size_t)qt * 8 * IA_WAVE * 16;  // KS = 4: NP = 8 h16x8 per lane
  return qfrag + NQ * 36 + (size_t)qt * 32 + (size_t)((qt + 3) & ~3) * 4 + (size_t)Mpad * 8;
}
int ia_launch_k3p(int qt, const void *db, const void *qf, const float4 *qinfo, const float4 *boxes, const int *pos2row,
                   int NT, int qt0, int M, int Mpad, int nwg, float4 *rec, float *recT, unsigned long long *pairs,
                   unsigned long long *tiles, int variant, int step, const int *ord_in, int n_in, int r0, int *ord_out,
                   const float4 *tbox, const float *tnorm, hipStream_t st, int nqb, int qt_end, const XOScan *xo,
                   unsigned long long *stamp, int rec_wt) {
  typedef k3p_fn (*getter)(int);
  static const getter g4[] = {ia_k3p_get_4_1, ia_k3p_get_4_2, ia_k3p_get_4_3, ia_k3p_get_4_4,  ia_k3p_get_4_5, ia_k3p_get_4_6,
                              ia_k3p_get_4_7, ia_k3p_get_4_8, ia_k3p_get_4_9, ia_k3p_get_4_10, ia_k3p_get_4_11};
  const int kmax = (NT + nwg - 1) / nwg;  // DB tiles per workgroup
  const int rev = step & 1;  // alternate steps walk in reverse
  // the in-kernel sort (20, 22, 24) holds <= 512 queries (wider: the host ran K2s, the presorted
  // form 21 / 25); every variant walks any number of tiles (the host keeps kmax <= IA_K3P_MAXK_LDS)
  const bool in_kernel_sort = variant == 20 || variant == 22 || variant == 24;
  if (in_kernel_sort && Mpad > 512) variant = 21;
  const size_t NQ = (size_t)qt * IA_TILE;
  const int nthr = IA_WGH;
  auto dyn_lds = [&](int v) {
    const bool pre = v == 21 || v == 25;
    const size_t qfrag = (size_t)qt * (v >= 24 ? 4 : 8) * IA_WAVE * 16;  // v24 / 25: hi pieces only
    size_t l = pre ? qfrag + NQ * 36 + (size_t)qt * 32 + (size_t)((qt + 3) & ~3) * 4 + NQ * 4 + (size_t)kmax * 40
                   : ia_k3p_lds(qt, Mpad) - (size_t)qt * 8 * IA_WAVE * 16 + qfrag + (size_t)Mpad * 4 + (size_t)kmax * 40;
    l += NQ * 8 + (size_t)kmax * 4;            // (z, w) per sorted query slot, R_t per tile
    if (v >= 24) l += (size_t)kmax * 8;        // the filter-passing tiles and their blocks
    size_t red = (size_t)(nthr / IA_WAVE) * qt * IA_TILE * 20;  // the subset merge's Top2 area
    if (v >= 24) red = std::max(red, (size_t)(nthr / IA_WAVE) * qt * IA_WAVE * 12);  // (every lane's subset)
    return l > red ? l : red;
  };
  size_t lds = dyn_lds(variant);
  if (variant >= 24) {  // the static LDS-DMA rings (86 KiB) + this launch's dynamic part must fit 160 KiB
    hipFuncAttributes fa;
    const k3p_fn f24 = g4[qt - 1](variant);
    const size_t stat = f24 && hipFuncGetAttributes(&fa, (const void *)f24) == hipSuccess ? fa.sharedSizeBytes : 0;
    // (and the second pass stages the lo pieces + a row map of the WG's tiles in the rings' 84 KiB)
    const bool ring_fits = (size_t)qt * 4 * IA_WAVE * 16 + (size_t)kmax * IA_TILE * 4 <= (size_t)8 * 3 * 3584;
    if (!f24 || !ring_fits || stat + lds > 160 * 1024) {  // (many tiles per workgroup or wide steps): the one-pass forms
      variant = variant == 25 ? 21 : 22;
      lds = dyn_lds(variant);
    }
  }
  const k3p_fn fn = g4[qt - 1](variant);
  // (the host accepts only the built variants, ia_set_option; a missing instance is an error the
  // level reports, never a silently skipped scan whose stale records the merge would consume)
  if (!fn) return -1;  // IA_EINVAL (include/ia.h)
  const bool pre = variant == 21 || variant == 25;
  // nqb > 1 (presorted variants only): one launch of nqb query blocks x nwg DB chunks
  if (!pre && !(xo && xo->on)) nqb = 1;
  if (nqb == 1) qt_end = qt0 + qt;
  XOScan x{};  // off unless an owner-computes step passes its exchange
  if (xo) x = *xo;
  x.stamp = stamp;
  x.rec_wt = rec_wt;
  allow_full_lds((const void *)fn);
  hipLaunchKernelGGL(fn, dim3(nqb * nwg), dim3(nthr), lds, st, (const h16x8 *)db, (const h16x8 *)qf, qinfo, boxes, pos2row,
                     NT, qt0, M, Mpad, nwg, rec, recT, pairs, tiles, rev, ord_in, n_in, r0, ord_out, tbox, tnorm, nqb, qt_end, x);
  return 0;
}
