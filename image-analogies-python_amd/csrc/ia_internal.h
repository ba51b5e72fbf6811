// ia_internal.h — shared host/device definitions of libia (MI355X / gfx950 only).
//
// Data layout in HBM:
//   * pyramid levels: row-major fp64 (h, w, ch), exactly the reference's arrays.
//   * feature DB of a level (create_index, algorithms.py:50-70): N_A rows of D = 55*ch
//     features, centred by a per-(part, channel) mean mu and stored fp32 together with the
//     row norm |a'|^2 in column D, zero padded to DP = 2*KH columns.  Rows are grouped in
//     tiles of 32 and each tile is stored in MFMA-fragment order:
//         float4 piece p (0..KH/4-1), lane L (0..63):  row  = tile*32 + (L & 31)
//                                                       cols = (L >> 5)*KH + 4p .. +3
//     so one wave loads a tile with KH/4 fully coalesced 1 KiB global_load_dwordx4.
//   * queries of a wavefront step use the same fragment order with values -2*q' and 1.0 in
//     column D, so one v_mfma_f32_32x32x2_f32 chain yields |a'|^2 - 2 q'.a' = |q-a|^2 - |q'|^2.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define IA_WAVE 64
#define IA_TILE 32          // DB rows per MFMA tile (M side of 32x32x2)
#define IA_WG 256           // threads per workgroup for every kernel
#define IA_MAX_D 168        // max padded feature width (3 channels: 165 + norm -> 168)
#define IA_WG_TARGET 512    // distance-kernel workgroups per step (2 per CU on 256 CUs)
#define IA_PAD_NORM 1.0e30f // norm of padding rows: never a candidate
#define IA_WGH 512          // threads per workgroup of the split-f16 distance kernel (8 waves)
#define IA_NWG_H 256        // its workgroups per step (1 per CU: the step's queries fill LDS)
#define IA_NORM_SCALE 256.0 // split-f16 DB stores |a'|^2 / 256 (query column D holds 256)
#define IA_F16_MAXABS 64.0  // split-f16 matcher only when every image value is within +-64

// Split-f16 DB tile in HBM (k_db_build_h): pieces p = 2s + part (part 0 = hi, 1 = lo) of
// 64 lanes x h16x8 in v_mfma_f32_32x32x16_f16 operand order.  When the upper half of the last
// k-step is pure padding (KS = 4: columns 56..63, D + 1 = 56), its two pieces store lanes 0..31
// only: 7 KiB instead of 8 KiB per tile, a 224 MiB 1024^2 DB that stays resident in the 256 MB
// memory-side cache across steps.  Upper-half lanes re-load the lower half's (finite) values:
// the query's columns there are zero, so those products are exact zeros.
template <int KS>
struct TileFmt {
  static constexpr bool CMP = KS == 4;
  static constexpr int STRIDE = CMP ? (2 * KS - 2) * IA_WAVE + 2 * IA_TILE : 2 * KS * IA_WAVE;  // h16x8 per tile
  __host__ __device__ static constexpr int off(int p, int L) {
    return (CMP && p >= 2 * KS - 2) ? (2 * KS - 2) * IA_WAVE + (p - (2 * KS - 2)) * IA_TILE + (L & 31) : p * IA_WAVE + L;
  }
};
// nearest-neighbour matcher of the distance scan (option "matcher")
#define IA_MATCH_F32 0      // v_mfma_f32_32x32x2_f32 on fp32 operands
#define IA_MATCH_F16X3 1    // v_mfma_f32_32x32x16_f16 x3 on hi/lo-split f16 operands

// feature descriptor: which image part, offset and channel
//   part 0: coarse 3x3 of A (level l-1)   part 1: fine 5x5 of A (level l)
//   part 2: coarse 3x3 of A'              part 3: first 12 of fine 5x5 of A'
struct FeatDesc {
  int8_t part, dy, dx, c;
};

struct LevelGeo {
  int ch, D, KH, n_ap;
  int KS;                   // split-f16 k-steps of 16 (0: fp32 matcher)
  int ah, aw, ahc, awc;     // A level l / l-1 dims
  int bh, bw, bhc, bwc;     // B level l / l-1 dims
  int64_t NA;               // DB rows = n_ap * ah * aw
  int n_tiles;              // ceil(NA / 32) over the whole DB
  int tile0, tile1;         // this rank's shard [tile0, tile1)
  int tiles_per_wg, nwg;    // distance-kernel decomposition of the shard
  const int *pos2row;       // pruned levels: position -> row table (ia_prune.hip); nullptr: ia_pos_row
};

struct Imgs {        // the four pyramid images a feature row reads (see FeatDesc parts)
  const double *p0;  // coarse (level l-1) of A or B
  const double *p1;  // fine (level l) of A or B
  const double *p2;  // coarse of A' or B'
  const double *p3;  // fine of A' or B'
  int h, w, hc, wc;  // fine / coarse dims
  int64_t img_stride_f, img_stride_c;  // per-A'-image strides (0 for B')
};

struct MergeArgs {
  const double *db64;  // fp64 row-major feature DB of the level (K1b), stride ia_db64_stride(ch)
  const float4 *rec;
  const float *recT;
  const double *q64;   // Mpad x D query rows (fp64)
  const double *qn2;   // |q'|^2 per query
  const unsigned *Rbits;
  int nwg, tpw;        // K3 decomposition of this rank's shard
  int pos0, pos_end;   // this rank's DB positions [tile0*32, tile1*32)
  int NT;              // tiles of the whole DB: position p holds row ia_pos_row(p, NT)
  int NA;              // DB rows
                                      // (per-pixel stats words, JobPtrs::pstat: bits 0-15
                                      // reranked, 16-28 fallbacks, 29 kappa decision ambiguous
                                      // under libm pow, 30 coherence won, 31 an MFMA value
                                      // outside the certified error bound)
  double eps_c;                      // relative error coefficient of the MFMA value
  double eps_a;                       // absolute (f16 subnormal) error coefficient
  const int *pos2row;                 // position -> row table (pruned levels) or nullptr
  int rr;                             // 1: workgroup w's chunk is tiles {w, w + nwg, ...} (pruned
                                      // scan); 0: the contiguous range [w*tpw, (w+1)*tpw)
  const float4 *qinfo;                // pruned levels: the step's query projection intervals (K2p)
  const float4 *boxes;                // pruned levels: per-tile projection boxes (ia_prune.hip)
  double ufac;                        // pruned levels: bound factor of ia_prune.h
  int img_rows;                       // 1: exact rows gathered from the A-side images (1 channel)
  // owner-computes sharded step (exchange = 2): records chunk-major in the exchange area (rec[w
  // xo_Mrec + m], (T, seq) in xo_rts), record w = chunk w mod xo_nch of shard w / xo_nch (storage
  // tiles ia_shard_off(NT, xo_W, s) + k + xo_nch i); boxes / pos2row are the whole level's
  const unsigned long long *xo_rts = nullptr;
  const int *xo_inv = nullptr;        // the owners' tables: query (o QTs 32 + local) -> slot
  int xo_W = 0, xo_nch = 0, xo_Mrec = 0, xo_o0 = 0, xo_M = 0, xo_QTs = 0;  // query m: owner xo_o0 + m / xo_M
  unsigned xo_seq = 0;
  unsigned *xo_err = nullptr;         // bit 3: a record did not arrive in time
  long long xo_timeout = 0;
  unsigned long long *stamp = nullptr;  // option "stamps": this launch's per-workgroup (start, end)
};

// Per-launch device timing without HIP events (option "stamps"): every workgroup of a stamped
// launch stores its (start, end) s_memrealtime ticks (100 MHz) at stamp[2 blockIdx], with vector
// stores from one lane; k_stamp_durations turns each launch's slots into max(end) - min(start).
// The timed, concurrent (pipelined) bench steps thereby report the device time of the kernels
// they actually ran.
__device__ __forceinline__ unsigned long long ia_clock() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ void ia_stamp_wg(unsigned long long *stamp, unsigned long long t0) {
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  stamp[2 * blockIdx.x] = t0 | 1ull;  // nonzero: a slot that was written (one tick of slack)
  stamp[2 * blockIdx.x + 1] = t1;
}

// DB positions are tile-strided and tile-scattered: slot j of tile t holds row j*NT + perm(t)
// with perm(t) = t * (IA_TILE_MUL mod NT) mod NT (a bijection: IA_TILE_MUL is a prime above any
// NT).  Spatially adjacent A pixels (near-identical features, near-tied distances) thereby land
// in different tiles AND far-apart tiles, i.e. in different K3 workgroup chunks: every chunk's
// runner-up threshold then stays clear of the winner and certification rarely needs an exact
// chunk rescan (with contiguous tiles, three near-ties of a smooth neighbourhood shared a chunk).
#define IA_TILE_MUL 2654435761LL
__host__ __device__ inline int64_t ia_tile_perm(int64_t t, int64_t NT) {
  const int64_t k = IA_TILE_MUL % NT;
  const int64_t p = t * k;  // < 2^52: exact in double
  int64_t q = (int64_t)((double)p / (double)NT);
  int64_t r = p - q * NT;
  r += r < 0 ? NT : 0;
  r -= r >= NT ? NT : 0;
  return r;
}
__host__ __device__ inline int64_t ia_pos_row(int64_t pos, int64_t NT) {
  return (pos & 31) * NT + ia_tile_perm(pos >> 5, NT);
}
__host__ __device__ inline int64_t ia_pos_row_t(int64_t pos, int64_t NT, const int *tab) {
  return tab ? (int64_t)tab[pos] : ia_pos_row(pos, NT);
}

// Pruned levels sharded over W ranks (ia_prune.hip k_make_table): Morton tile m belongs to
// shard m mod W; storage tile ts of shard r (storage range [off_r, off_r + NT_r), NT_r =
// ceil((NT - r) / W), off_r = r q + min(r, NT mod W), q = NT / W) holds Morton tile r + W k.
__host__ __device__ inline int64_t ia_shard_morton_tile_(int64_t ts, int64_t NT, int W) {
  const int64_t q = NT / W, rem = NT % W;
  int64_t r, k;
  if (ts < rem * (q + 1)) {
    r = ts / (q + 1);
    k = ts - r * (q + 1);
  } else {
    r = rem + (ts - rem * (q + 1)) / q;
    k = ts - rem * (q + 1) - (r - rem) * q;
  }
  return r + (int64_t)W * k;
}
__host__ __device__ inline int64_t ia_shard_off(int64_t NT, int W, int r) { return r * (NT / W) + (r < NT % W ? r : NT % W); }

// certified pruning of the distance scan (ia_prune.hip): projection basis size, smallest DB
// that prunes
#define IA_NPC 4
#define IA_PRUNE_MIN_ROWS 524288  // default of option "prune_min_rows": at 512^2 (262,144 rows) the
                                  // unpruned scan + cheaper gather/merge is still faster
// DB tiles per workgroup the pruned scan takes (its tile boxes, need masks and R_t in LDS: 44 B
// per tile next to <= 11 query tiles); larger DBs (> 8.4 M rows per shard) scan unpruned
#define IA_K3P_MAXK_LDS 1024

// per-step wavefront description: pixels (r, t - 3r), r in [r0, r0 + M), of each of J jobs.
// Query m of the step (0 <= m < J*M) is job m / M, row r0 + m % M; Mpad = J*M rounded up to
// whole query tiles of 32.
struct StepDesc {
  int t, r0, M, Mpad, J;
};

// One synthesis job of a batched level (ia_synthesize_levels): its B side.  Every job of a
// batch shares the level's A side (one DB) and the B level shape, so the wavefront steps align.
#define IA_MAX_JOBS 32
struct JobPtrs {
  const double *Bc, *B, *Bpc;  // B level l-1, l and B' level l-1 (complete)
  double *Bp;                  // B' level l: in init, out synthesised
  int32_t *s, *im;             // source maps (written)
  unsigned *pstat;             // per-pixel stats words of the level
  int32_t *dbg_src;            // optional debug records (include/ia.h), nullptr: off
  double *dbg_dist;
  const double *weights;       // compute_distance weights
  double kf;                   // kappa factor 1 + 2^(level - L) k
  int32_t *nn;                 // option "nn_bound" (pruned one-rank levels): per pixel the row of its
                               // certified exact NN (-1: none yet), written by the merge; the gathers
                               // shift the causal neighbours' rows into extra U' candidates (nullptr: off)
};
// the jobs of a launch.  A single job (the common case) travels in the kernel arguments
// (JobArg1: its pointers are plain kernel-argument loads, as before batching); a batch reads
// them from a device array with a wave-uniform index (JobArgN).  The kernels are templated on
// the two, so neither pays for the other (a runtime select between a by-value argument and a
// global array made the compiler spill the argument to LDS and read every pointer with flat
// loads: +5 us per K2p launch).
struct JobArg1 {
  static constexpr bool single = true;  // the launcher also puts its images into the Imgs argument
  JobPtrs j0;
  __device__ __forceinline__ JobPtrs get(int) const { return j0; }
};
struct JobArgN {
  static constexpr bool single = false;
  const JobPtrs *rest;
  __device__ __forceinline__ JobPtrs get(int job) const { return rest[job]; }
};
struct JobSet {   // host side: what the launchers dispatch on
  JobPtrs j0;
  const JobPtrs *rest;  // device JobPtrs[n_jobs]
  int J;
};
struct QPix {
  int job, r, c, qi;           // job, pixel (r, c) and its raster index in the B level
};
__host__ __device__ inline QPix ia_qpix(const StepDesc &sd, int bw, int m) {
  QPix p;
  p.job = m / sd.M;
  p.r = sd.r0 + (m - p.job * sd.M);
  p.c = sd.t - 3 * p.r;
  p.qi = p.r * bw + p.c;
  return p;
}

// single-rank certified winner of one query
struct Winner {
  double d;
  int64_t idx;
};

// One-shot peer-write winner exchange of a sharded level (option "exchange" = 1):
// every rank's exchange buffer holds, per step parity (2) x rank (W) x query (IA_XCHG_MAXQ), a
// 16-byte slot: the certified shard winner's exact distance, then (row | step sequence << 32)
// written once the distance store has completed (ia_stores_done; the buffer is uncached).  The merge of each rank writes its
// winner into the slot of every peer (xGMI stores into the peers' buffers, opened through HIP
// IPC handles) and polls its own buffer for the W winners of the step.  Two parities suffice: a
// rank can be at most one step ahead of any peer (its step t+1 needs every step-t winner).
#define IA_XCHG_MAXQ 4096  // queries per step (>= the widest 1-job step: min(h, ceil(w / 3)))
#define IA_XCHG_MAXW 16    // ranks of one exchange
struct XSlot {
  double d;
  unsigned long long row_seq;  // row (low 32 bits) | sequence number (high 32 bits)
};
struct XchgArgs {
  XSlot *peer[IA_XCHG_MAXW];   // every rank's exchange buffer in this process's address space
  XSlot *local;                // this process's buffer (polled)
  int W, rank;                 // ranks (shards) and the shard this launch publishes as
  unsigned seq;                // exchange sequence number of the step (identical on every rank)
  unsigned *err;               // bit 0: a peer's winner did not arrive in time
  long long timeout_ticks;     // s_memrealtime ticks (100 MHz) before giving up
};
__host__ __device__ inline size_t ia_xslot(unsigned seq, int W, int rank, int m) {
  return ((size_t)(seq & 1u) * W + rank) * IA_XCHG_MAXQ + m;
}

// Owner-computes sharded steps (option "exchange" = 2): W ranks, rank o owns job o
// (its gather K2p, query sort K2s and merge K4 run there only) and every rank scans ITS DB shard
// for the queries of all W jobs.  Two one-shot exchanges per wavefront step through each rank's
// exchange area (after the winner slots of the same IPC buffer; two parities, seq & 1):
//   * owner o's K2s writes its job's sorted query tiles (fragments, pruning records, tile boxes,
//     slot -> query map) at tiles [o QTs, o QTs + QTs) of EVERY rank's area, then per tile a
//     flag = seq (after a system-scope fence); each K3p workgroup polls its block's tile flags;
//   * K3p workgroup (block b, chunk k) of shard s writes the records of its block's queries into
//     owner b's area, chunk-major in sorted-slot order (record w = s nch + k of slot x at w Mrec +
//     x: one contiguous 1 KiB store per wave-instruction over xGMI), float4 (v1, row1, v2, row2)
//     then, after a system-scope fence, (T, seq); the owner's fused merge K4 finds a query's slot
//     in its own table (written by its K2s into local memory) and polls each record's seq.
// No winner exchange and no finish: the owner's K4 is the single-GPU merge over W nch records
// per query.  Every rank holds the whole DB (the fp64 rows a rerank or rescan needs), 0.7 GB per
// 1024^2 level.
// Ordering of an exchange hand-off: the payload goes to uncached memory (nothing in any L2 to
// write back), so the writer waits for its own stores' completion (s_waitcnt vmcnt(0): a store
// to uncached memory completes at the memory side) before the flag / seq store - no system-scope
// release fence, whose L2 write-back of every dirty line costs microseconds per wave.
__device__ __forceinline__ void ia_stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
#define IA_XO_MAXT 128            // query tiles of a step over all owners (4096 queries)
#define IA_XO_MAXREC (1 << 20)    // records of a step over all owners' queries (W nch per query)
struct XOLayout {                 // byte offsets inside one parity of an exchange area (KS = 4 fragments)
  static constexpr size_t FRAG = 0;                                   // [tile][8][64] h16x8
  static constexpr size_t INFO = FRAG + (size_t)IA_XO_MAXT * 8 * 64 * 16;  // [slot][3] float4
  static constexpr size_t TBOX = INFO + (size_t)IA_XO_MAXT * 32 * 48;      // [tile][3] float4
  static constexpr size_t ORD = TBOX + (size_t)IA_XO_MAXT * 48;            // [slot] int: query of the owner
  static constexpr size_t FLAG = ORD + (size_t)IA_XO_MAXT * 32 * 4;        // [tile] unsigned seq (K2s path)
  static constexpr size_t QSEQ = FLAG + (size_t)IA_XO_MAXT * 4;            // [slot] unsigned seq (K2p path)
  static constexpr size_t REC = QSEQ + (size_t)IA_XO_MAXT * 32 * 4 + 256;  // [w][Mrec] float4
  static constexpr size_t RTS = REC + (size_t)IA_XO_MAXREC * 16;           // [w][Mrec] (T bits, seq)
  static constexpr size_t PARITY = RTS + (size_t)IA_XO_MAXREC * 8;
};
__host__ __device__ inline size_t ia_xslots_bytes(int world) { return (size_t)2 * world * IA_XCHG_MAXQ * sizeof(XSlot); }
// what K2s of an owner writes: every rank's area of this parity (W of them; 1 when emulated:
// one area serves every shard)
struct XOSort {
  char *area[IA_XCHG_MAXW];       // parity base of each rank's area
  int *inv;                       // the owner's own table (local memory): inv[tile0 32 + query] = slot
  int W;                          // areas written
  int q0, Mj;                     // the owner's queries in the local K2p output: [q0, q0 + Mj)
  int tile0, QTs;                 // its tiles in the step layout [tile0, tile0 + QTs)
  unsigned seq;
};
// Owners whose step fits one launch's query tiles (<= 352 queries: cfg3) skip K2s: their K2p
// publishes its unsorted queries (fragments, pruning records) at slots [slot0, slot0 + Mpad_j)
// of every rank's area, each followed by its seq, and every K3p block sorts its owner's queries
// itself (the single-GPU in-kernel sort); the scan of the owner's own shard writes its table.
struct XOPub {
  char *area[IA_XCHG_MAXW];       // parity base of each rank's area (emulated: 1, local)
  int W, slot0;                   // areas written; the owner's first slot
  unsigned seq;
};
// what K3p needs besides its query inputs (which point into the local area)
struct XOScan {
  char *area[IA_XCHG_MAXW];       // parity base of each owner's area (emulated: every entry local)
  const unsigned *flag;           // local area's tile flags (PRE) or per-slot seqs (in-kernel sort)
  int *inv;                       // in-kernel sort: the owner's table (written by the owner's shard)
  int on, s, bpj;                 // owner of block b = b / bpj; this launch scans shard s
  int Mrec;                       // record rows per chunk (slots of the step layout)
  unsigned seq;
  unsigned *err;                  // bit 2: a tile flag did not arrive in time
  long long timeout_ticks;
  unsigned long long *stamp;      // option "stamps" (any K3p launch, owner-computes or not): per-WG ticks
  int rec_wt;                     // option "rec_wt": records stored write-through (sc1), nothing left dirty in L2
};

// fused K4(t) + K2p(t + 1) (k_merge_gather, option "fuse_gather"): the next step's gather
// outputs (the other parity half of the query buffers) and the per-row handoff slots
struct HandSlot {          // uncached: row r's step-t result for row r + 1's step-(t + 1) query
  double v;                // B' value
  int sr, sc, im;          // source pixel, A' image
  unsigned seq;            // the step's seq, stored after the fields above completed
  int nn;                  // its exact NN row (option "nn_bound"; -1: none)
  unsigned pad;
};
struct NextStep {
  StepDesc sn;             // step t + 1
  const double *mu, *basis;
  double *q64, *qn2;
  void *qf;
  float4 *qinfo;
  double ufac;
  HandSlot *hand;          // one slot per B row
  unsigned seq;
  unsigned *err;           // bit 4: a handoff did not arrive in time
  long long timeout_ticks;
  XOPub xp;                // owner-computes step t + 1: publish its queries (xp.W = 0: off)
  const unsigned *wait_seq;  // owner-computes ranks: one extra wave waits until all wait_n query
  int wait_n;                // seqs of step t + 1 (this rank's area) arrived, so the next scan
                             // starts with its queries in place instead of spinning on every CU
  // option "fuse_sort" (pruned one-rank levels): the gathers of step t + 1 also sort it for the
  // presorted scan.  Every gather wave publishes its query's sort key with the step's seq
  // (kslot[m], uncached), waits until all sn.Mpad keys of the step are there, counts the keys
  // below its own (its sorted slot x) and writes its pruning record, fragments and query index
  // at slot x (sinfo / sfrag / sorder: k_query_sort's outputs); the scan then skips its
  // per-workgroup sort (kslot = nullptr: off)
  unsigned long long *kslot;
  int prefetch;              // option "prefetch_next": the gathers' step-independent inputs load during the merge
  int early;                 // option "early_gather": the merge waves' gathers run everything but the row
                             // above's feature before its handoff (ia_kernels.hip gather_p_early)
  int *sorder;
  float4 *sinfo;
  void *sfrag;
};

__host__ __device__ inline int ia_reflect(int i, int n) {
  // np.pad(mode='symmetric') index map (img_preprocess.py:81-83).  Windows reach at most 2
  // pixels past an edge, so two folds suffice unless the image is narrower than the window;
  // only then take the (slow, integer-modulo) periodic form.
  int j = i < 0 ? -i - 1 : i;
  j = j >= n ? 2 * n - 1 - j : j;
  if ((unsigned)j < (unsigned)n) return j;
  const int m = 2 * n;
  i %= m;
  if (i < 0) i += m;
  return i >= n ? m - 1 - i : i;
}

// error bound of the fp32 MFMA value |a'|^2 - 2q'.a' against exact arithmetic:
//   |err| <= gamma_n * (|a'|^2 + 2 sum|q'_k a'_k|) <= gamma_n * (R^2 + 2 R |q'|),  n = DP + 2
// with u = 2^-24, gamma_n = n u / (1 - n u); 5% margin on top.
inline double ia_eps_c(int DP) {
  const double nu = (DP + 2) * 5.9604644775390625e-08;
  return 1.05 * nu / (1.0 - nu);
}

// Split-f16 MFMA value: x = a' or |a'|^2/256, y = -2q' or 256, each split as
// hi = f16(f32(x)), lo = f16(f32(x) - hi); the kernel sums hi*hi + lo*hi + hi*lo (exact f16
// products) in fp32 over n <= 48*KS + 4 terms.  Per term |x*y - computed| <= 3.5*2^-22 |x y| +
// 2^-25 (|x| + |y|) (representation + dropped lo*lo; 2^-25 = half the f16 subnormal spacing),
// and the fp32 accumulation, whatever its internal order or rounding (round-to-nearest or
// truncation, hence u = 2^-23), adds gamma_n * sum|terms|.  With sum|x y| <= R^2 + 2R|q'| and
// sum(|x| + |y|) <= R^2/256 + sqrt(D)(R + 2|q'|) + 256 + 1 (D <= 176):
//   eps = eps_c (R^2 + 2R|q'|) + eps_a (R^2 + 14 R + 28|q'| + 260)
// packed: the packed-index K3h epilogue replaces each value's 4 low mantissa bits by a row
// index, moving it by < 16 ulp <= 2^-19 |v| <= 2^-19 (R^2 + 2R|q'|) (1 + 1e-2 headroom).
inline double ia_eps_c_h(int KS, bool packed) {
  const double nu = (48.0 * KS + 4) * 1.1920928955078125e-07;
  return 1.05 * (nu / (1.0 - nu) * (1.0 + 1.0 / 512) + 3.5 * 2.384185791015625e-07) +
         (packed ? 1.01 * 1.9073486328125e-06 : 0.0);
}
inline double ia_eps_a_h() { return 1.05 * 2.9802322387695312e-08; }
