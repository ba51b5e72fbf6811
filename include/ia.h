/*
 * ia.h — C ABI of the MI355X-native Image Analogies best-match core (libia.so).
 *
 * The reference (flair2005/image-analogies-python) reaches native code in exactly one place:
 * pyflann, a ctypes shim over libflann's C ABI, called from algorithms.py:56 (pf.FLANN()),
 * algorithms.py:69 (build_index) and algorithms.py:74 (nn_index).  Everything else on the hot
 * path is the Python raster loop image_analogies.py:130-239.  This header replaces both:
 *
 *   ia_index_*            drop-in for the FLANN object API (algorithms.py:56,69,74):
 *                         build an exact-NN index over caller rows, query it in batches.
 *   ia_synthesize_level   drop-in for one iteration of the per-level loop
 *                         (image_analogies.py:130-239 incl. create_index's DB for that level,
 *                         algorithms.py:50-70): DB build, skewed-wavefront schedule, exact NN,
 *                         coherence, kappa selection and B'/s/im writeback, all on the GPU.
 *
 * Conventions (pyflann's, kept): caller-owned C-contiguous buffers, library-owned opaque
 * handles, integer status returns (0 = ok, negative IA_E* on error, never throws across the
 * ABI), thread-local ia_last_error().  Images are row-major (h, w[, ch]) fp64 in [0,1] scale
 * exactly as the reference keeps them; index outputs are int32/int64.
 * A context is not thread-safe; one host thread drives one context (one GPU).
 */
#ifndef IA_H_
#define IA_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IA_OK 0
#define IA_EINVAL -1   /* bad argument / shape contract violated */
#define IA_EHIP -2     /* HIP runtime error */
#define IA_ENOMEM -3   /* device allocation failed */
#define IA_ENODEV -4   /* no usable gfx950 device */
#define IA_ECOMM -5    /* RCCL error */

#define IA_MEM_HOST 0   /* pointers in ia_level_args are host (numpy) memory */
#define IA_MEM_DEVICE 1 /* pointers are device memory already resident in HBM */

typedef struct ia_ctx ia_ctx;
typedef struct ia_index ia_index;

/* Per-call statistics (SURVEY §5 'Metrics'). */
typedef struct {
  int64_t pixels;          /* B' pixels synthesised */
  int64_t steps;           /* wavefront steps executed */
  int64_t coherence_wins;  /* pixels whose source came from best_coherence_match */
  int64_t reranked;        /* exact fp64 reranks of MFMA candidates */
  int64_t fallbacks;       /* uncertified DB chunks rescanned exactly */
  double db_ms;            /* DB build time (device) */
  double synth_ms;         /* wavefront time (device) */
  int64_t dist_launches;   /* MFMA distance kernel launches */
  double dist_flops;       /* algorithmic flops 2*D*N_A*(queries) of those launches */
  /* sampled timing of the MFMA distance kernel (option "time_dist" = sampling stride S > 0:
   * every S-th wavefront step's distance launches are bracketed by HIP events) */
  double dist_ms;          /* device time of the sampled launches */
  int64_t dist_launches_timed;
  double dist_flops_timed; /* algorithmic flops of the sampled launches */
  int64_t bound_violations; /* pixels where a reranked candidate's exact distance fell outside
                             * the certified MFMA error bound (audit; expected 0) */
  int64_t f16_levels;       /* levels run on the split-f16 matcher */
  int64_t pruned_levels;    /* levels run on the certified pruned scan (option "prune") */
  double dist_pairs;        /* (DB tile, query tile) pairs the distance kernel contracted */
  double dist_pairs_full;   /* pairs an unpruned scan contracts (dist_pairs / this = work left) */
  double dist_tiles;        /* DB tiles the distance kernel loaded (summed over its launches) */
  double dist_tiles_full;   /* DB tiles an unpruned scan loads (dist_tiles / this = DB bytes left) */
  double prune_ms_timed;    /* pruned-scan launches of the timed steps (option "time_dist"): device ms */
  int64_t prune_launches_timed;
  double prune_flops_timed; /* their MFMA flops (computed pairs x 2 D 32 32) */
  double prune_bytes_timed; /* their algorithmic bytes (DB tiles loaded, boxes, queries, records) */
  int64_t kappa_ambiguous;  /* pixels whose kappa decision (image_analogies.py:206) would flip if
                             * compute_distance's `** 2` (libm pow on a numpy scalar) rounded a
                             * near-midpoint square the other way than y * y does (audit; no
                             * fixture has one) */
  double dist_pairs_corrected; /* k3p_variant 14/15: pairs whose hi x hi value passed the bound
                                * (correction products + top-2 epilogue run); 16/17: pairs whose
                                * head (15-axis partial distance) passed; else 0 */
  double dist_tiles_rows;   /* hi x hi block filter (k3p_variant 14, 15, 18..21): loaded DB tiles with
                             * at least one block passing the filter (the only ones whose lo halves
                             * the correction products read) */
  /* feature-gather kernels (bench.py roofline.gathers; DESIGN.md §4 algorithmic bytes) */
  double k1b_ms;            /* K1b k_db64_build (fp64 row DB), device ms summed over the levels */
  double k1b_bytes;         /* its algorithmic bytes: A-side images read once + N_A rows written */
  double k1_ms;             /* K1 k_db_build_h (split-f16 tiles), device ms summed over the levels */
  double k1_bytes;          /* its algorithmic bytes: fp64 rows read + tiles written */
  int64_t build_levels;     /* levels summed in k1*_ms / k1*_bytes: those with the largest DB
                             * (build_rows) this ia_stats has seen (the bench's finest level) */
  double gather_ms_timed;   /* K2 (k_gather_query_*) of the sampled steps ("time_dist"): device ms */
  int64_t gather_launches_timed;
  double gather_bytes_timed; /* their algorithmic bytes: 55 features + 12 coherence rows read,
                              * fp64 row + fragments + pruning record written per query */
  double merge_ms_timed;    /* K4 (k_merge_level) of the sampled steps: device ms */
  int64_t merge_launches_timed;
  int64_t build_rows;       /* DB rows of the levels in k1*_ms (the largest seen) */
  /* option "stamps" = 1: device time of EVERY pruned-scan launch and every fused merge launch of
   * the pruned levels, from per-workgroup s_memrealtime stamps written by the kernels themselves
   * (no HIP events, nothing on the stream between kernels: valid in pipelined / concurrent runs) */
  double k3p_stamp_ms;      /* summed over the launches: max(WG end) - min(WG start) each */
  int64_t k3p_stamp_launches;
  double k3p_bytes_all;     /* algorithmic bytes of those launches (tiles loaded, boxes, queries, records) */
  double merge_stamp_ms;    /* the merges (k_merge_gather / fused k_merge_level) of the same levels */
  int64_t merge_stamp_launches;
  double stamp_gap_ms;      /* one-job levels: idle time between the chain's kernels (scan end -> merge
                             * start, merge end -> next scan start), summed */
  int64_t stamp_gaps;
  double stamp_window_ms;   /* those levels' first scan start -> last kernel end */
  int64_t prune_rows;       /* DB rows of the pruned levels in prune_*, k3p_*, merge_stamp_* and
                             * stamp_* (the largest pruned level seen: the bench's finest) */
  double k3p_stamp_start_ms; /* the same K3p launches: last workgroup start - first start, summed */
  double k3p_stamp_wg_ms;    /* ... their mean workgroup duration (end - start), summed */
  double stamp_gap_sm_ms;   /* the scan end -> merge start part of stamp_gap_ms */
  int64_t stamp_gaps_sm;
  double k3p_bytes_unique_all; /* k3p_bytes_all with each launch's DB tiles counted at most once
                                * (<= the launch's whole tiles): launches of several query blocks
                                * stream a tile once per block (cfg4's wide steps) */
} ia_stats;

/* One pyramid level (image_analogies.py:130-239).  Shapes: A/A' level l is (a_h, a_w[, ch]),
 * level l-1 is (ceil(a_h/2), ceil(a_w/2)[, ch]); same for B.  Ap / Apc stack n_ap images.
 * Bp: in = initial B' level (initialize_Bp, img_preprocess.py:66-78), out = synthesised.
 * s_out (N x 2, row/col in A) and im_out (N) are the reference's s / im lists for this level. */
typedef struct {
  int ch;          /* channels per pixel: 1 (luminance / grayscale) or 3 */
  int n_ap;        /* number of A' images (Ap_fname_list) */
  int a_h, a_w;    /* A level l */
  int b_h, b_w;    /* B level l */
  const double *A, *Ac;     /* A level l, l-1 (already AB_weight-compressed, image_analogies.py:65) */
  const double *Ap, *Apc;   /* A' level l, l-1, n_ap stacked */
  const double *B, *Bc;     /* B level l, l-1 (compressed) */
  const double *Bpc;        /* B' level l-1, complete */
  double *Bp;               /* B' level l: in init, out synthesised */
  const double *weights;    /* compute_distance weights (config.py:68-79), 55*ch */
  double kappa_factor;      /* 1 + 2^(level - max_levels) * k   (image_analogies.py:206) */
  int32_t *s_out;           /* N x 2 */
  int32_t *im_out;          /* N */
  int mem;                  /* IA_MEM_HOST or IA_MEM_DEVICE for every pointer in this struct */
  /* Optional debug structures of image_analogies_main(debug=True) (image_analogies.py:141-153,
   * 224-240); both NULL (off) or both given, single-rank levels only.  Per raster pixel:
   * dbg_src  N x 6 int32: p_app row, col, image (the NN, Ap_ix2px of best_approximate_match),
   *          r_star row, col (best_coherence_match, algorithms.py:126-130; 0, 0 without one),
   *          has_coh (1 when a coherence candidate existed, i.e. the kappa rule compared);
   * dbg_dist N x 2 fp64: v_app, v_coh = x.dot(x) of compute_distance's x = (a - q) * w
 *          (algorithms.py:133-135) in the golden host's BLAS order; 0 when has_coh = 0.
 *          compute_distance itself is np.sqrt(v) ** 2 with libm's pow (numpy scalar power),
 *          which is not always v's correctly rounded square root squared: the host applies it. */
  int32_t *dbg_src;
  double *dbg_dist;
} ia_level_args;

/* ---- context ---------------------------------------------------------------------------- */
int ia_init(int device, ia_ctx **out);
void ia_destroy(ia_ctx *ctx);
const char *ia_last_error(void);
int ia_version(void);
/* Options: "time_dist" = S (0 = off): bracket the MFMA distance launches of every S-th
 * wavefront step with HIP events; ia_stats.dist_ms / dist_flops_timed then give the kernel's
 * measured device time and algorithmic flops (bench.py roofline).
 * "matcher" = IA_MATCH_F16X3 (default: split-f16 MFMA scan, 1 and 2 channels, image values
 * within +-64) or IA_MATCH_F32 (fp32 MFMA scan).  Both are certified exact: identical results.
 * "prune" = 1 (default) / 0: certified pruned scan on 1-channel split-f16 levels with at least
 * "prune_min_rows" DB rows (default 2^19): (DB tile, query tile) pairs a
 * projection bound proves farther than the query's best coherence candidate are skipped.
 * "k3p_variant" / "k3_variant": kernel versions of DESIGN.md §4b / §4h / §4i; the product build
 * accepts k3p_variant 24 (default: the pruned scan sorts a step's queries itself up to 512 of
 * them, then runs two passes: every wave streams the hi halves of its DB tiles into LDS by
 * LDS-DMA, two tiles in flight, and runs the hi x hi block filter on the box-needed blocks;
 * then the tiles with a block that can lie within its query's bound get their full products +
 * top-2, handed out over the workgroup's waves; a step wider than 512 queries is sorted once by
 * k_query_sort and runs 21), 25 (24 presorted), 22 (one pass: the hi stream in registers, the
 * passing tiles' lo halves one tile later), 20 (whole tiles; 21 presorted) and k3_variant 1.
 * The other versions of DESIGN.md §4b / §4f are in git history.
 * "k3p_blocks" = 1 (default) / 0: a presorted pruned scan wider than one launch's 11 query tiles
 * runs as ONE launch of (query block x DB chunk) workgroups instead of one launch per block.
 * "fuse_gather" = 1 (default) / 0: on one-job unsharded pruned levels the merge of step t and the
 * gather of step t + 1 run as one launch (the step's results handed row to row through uncached
 * slots); 0 = separate launches.
 * "pipeline_last" = 1: the next level call has no dependents, so it records no per-step events
 * (level pipelining's finest level; applies to one call).
 * "stream_priority" = 0 (default) / 1 (high) / 2 (low): recreate the context's stream with that
 * priority (idle contexts; level pipelining puts the finest level's stream high).
 * "prune_group" = G in {1 (default), 2, 4, 8}: pruned levels store each group of G Morton tiles
 * interleaved (sort neighbours in different tiles and scan chunks: fewer certification rescans,
 * looser tile boxes).
 * "row_source" = 0 (exact rows of the rerank / coherence / pruning bound from the fp64 row DB);
 * 1 (gathered from the A-side pyramid images; measured slower) is in git history only.
 * "shard_emulate" = W (1 = off): on a single-rank context, every level with >= 64 W DB tiles
 * runs as a W-way DB shard on this device (per-shard scans and certified winners, then the
 * multi-rank finish; no RCCL): the sharded code path, testable on one GPU.
 * "shard_unpruned" = 0 (default) / 1: shard only the levels that run the pruned scan / every
 * level with >= 64 W tiles.  "exchange" = 0 (RCCL all-gather + finish) / 1 (peer-write merge)
 * / 2 (owner computes: each rank brings its own job, every rank scans its shard for all of them,
 * queries and scan records exchanged by peer writes; emulated: one job per shard).
 * "nn_bound" = 1 (default) / 0: on all pruned levels (every merge form: one-rank, sharded,
 * peer-write, owner-computes) the merge also keeps each pixel's certified
 * exact NN row, and the gathers bound U' (the pruned scan's radius) by the causal neighbours' NN
 * rows shifted by the neighbour's offset as well as by the coherence candidates (exact either way:
 * any DB row's exact distance bounds the NN distance).
 * "prefetch_next" = 1 (default) / 0: a fused merge + gather wave loads its next query's inputs
 * that do not depend on the launch's own merges (features, causal neighbours' sources) while
 * its merge's DB rows load.
 * "fuse_sort" = 0 (default) / 1 / 2: the fused gathers of step t + 1 also rank its queries' sort
 * keys across the launch and write the presorted scan inputs (no K2s launch, no per-workgroup
 * sort in the scan).  2: only on levels whose widest step has >= 512 queries (all jobs).  Exact
 * either way; no faster since option nn_bound.
 * Fused merge + gather launches (option "fuse_gather") wait row to row; a level uses them only
 * while the chained waves of all levels in flight in the process stay under twice the GPU's
 * resident k_merge_gather waves (else it runs separate launches; ia_capi.cpp g_chain_waves).
 * "rec_wt" = 1 (default) / 0: the pruned scan stores its per-(query, chunk) records write-through
 * (sc1 buffer stores), so the scan -> merge kernel boundary has no dirty record lines to write
 * back (one-rank steps; the owner-computes exchange has its own uncached stores).  Exact either
 * way: the merge reads the records after the boundary.
 * "early_gather" = 1 (default) / 0: a fused merge + gather wave of a one-rank pruned level (option
 * prefetch_next on, no publish) runs its next query's gather up to the row above's late feature
 * before waiting for that handoff: the other 54 features, fragments, projection and |q'|^2 sums,
 * and U' over the candidate rows requested first; U' then leaves out the row above's own two
 * candidates (a valid bound either way).
 * "scan_wgs" = 8..256 (a multiple of 8; default 256, one per CU): workgroups of the context's
 * split-f16 scans (pruned: one chunk of DB tiles each; unpruned: contiguous tile ranges).  bench.py
 * gives the coarser pipelined levels' contexts 128, so their scans never queue for the whole GPU
 * while the finest level's kernels are dispatched.
 * "stamps" = 1: every pruned-scan and fused-merge launch of a pruned level stamps its
 * workgroups' first / last s_memrealtime tick; ia_stats.k3p_stamp_ms / merge_stamp_ms sum the
 * per-launch device times (bench.py roofline.frac_timed: the timed, pipelined steps' own kernels).
 * "xo_presort" = 1: owner-computes steps always sort in a K2s launch (tests; default 0: steps of
 * <= 352 queries per owner are sorted inside the scan).  Environment IA_CU_SPLIT=k/n (rehearsals
 * of n ranks on ONE GPU only): the context's stream runs on CU slice k of n.
 * Identical results for every setting. */
#define IA_MATCH_F32 0
#define IA_MATCH_F16X3 1
int ia_set_option(ia_ctx *ctx, const char *name, int value);
/* Multi-GPU (one process per GPU): A rows of every level are split into `world` contiguous
 * shards; per wavefront step each rank exchanges its certified per-query winners with one
 * RCCL all-gather and every rank picks the same global winner (lowest index on ties).
 * ia_comm_unique_id fills 128 bytes on rank 0; broadcast them (torch.distributed) and call
 * ia_comm_init on every rank. */
int ia_comm_unique_id(unsigned char id_out[128]);
int ia_comm_init(ia_ctx *ctx, int rank, int world, const unsigned char id[128]);
/* One-shot peer-write exchanges for sharded levels (replace the RCCL all-gather +
 * finish of ia_comm_init).  Every rank calls ia_xchg_alloc (an uncached device buffer, zeroed:
 * 2 x world x 4096 16-byte winner slots for "exchange" = 1, then two parities of the owner
 * areas of "exchange" = 2, about 50 MiB) and publishes the returned 64-byte HIP IPC handle;
 * after gathering all world handles (rank order, world x 64 bytes) it calls ia_xchg_open, which
 * maps the peers' buffers and makes the context a rank of a world-rank DB shard (option
 * "exchange" = 1 unless 2 was set before).  No RCCL communicator is needed.  A peer that stops
 * publishing makes the level fail with IA_ECOMM after 20 s instead of hanging.  With option
 * "shard_emulate" = W and "exchange" = 1 / 2 a single process runs the same kernels over a
 * local buffer.  Every ia_xchg_open needs its own ia_xchg_alloc before the handle swap (a reused
 * buffer is zeroed there and the step sequence restarts on every rank alike; ia_comm_init
 * afterwards drops the peer mappings and returns to "exchange" = 0).  The ranks of one
 * exchange run the same sequence of level calls with identical A levels and identical B shapes
 * (per level): slots and sequence numbers are laid out from the local geometry, so ranks that
 * disagree time out (IA_ECOMM after 20 s) - check the shapes on the host first. */
int ia_xchg_alloc(ia_ctx *ctx, int world, unsigned char handle_out[64]);
int ia_xchg_open(ia_ctx *ctx, int rank, int world, const unsigned char *handles);

/* ---- fast path: one level ----------------------------------------------------------------- */
int ia_synthesize_level(ia_ctx *ctx, const ia_level_args *args, ia_stats *stats);
/* The same level for n_jobs independent jobs at once (multi_script.py's parameter sweeps,
 * multi_script.py:13-32: kappa / pyramid depth change, the A side does not).  args[0..n_jobs)
 * must share the A side (identical A, Ac, Ap, Apc pointers: one feature DB is built) and every
 * shape, channel count and mem kind; B, Bc, Bpc, Bp, weights, kappa_factor, outputs and debug
 * buffers are per job.  Every wavefront step gathers the queries of all jobs and runs ONE
 * distance scan over the DB for them (the DB is streamed once per step, not once per job), then
 * each job's coherence / kappa / writeback.  Results are those of n_jobs separate
 * ia_synthesize_level calls, bit for bit.  1 <= n_jobs <= 32.  Sharded levels take batches too
 * ("exchange" 0 / 1: every rank holds every job; emulated "exchange" = 2: one job per shard). */
int ia_synthesize_levels(ia_ctx *ctx, const ia_level_args *args, int n_jobs, ia_stats *stats);

/* Level pipelining: level l + 1 of a job only reads B' of level l near
 * (r / 2, c / 2), so its wavefront step t needs level l's steps <= t / 2 + 4, not the whole level.
 * Two contexts driven from two host threads run alternate levels concurrently: the context of
 * level l has option "pipeline_record" = 1 (its level calls are numbered 1, 2, ...: generations,
 * ia_pipeline_generation = the last one started) and before the level l + 1 call the other
 * context calls ia_pipeline_depend(ctx, prev_ctx, generation of level l): each of its steps then
 * waits (a stream event wait, no host sync) for the steps of level l it reads.  Results are those
 * of the sequential order, bit for bit.  A previous level that stops for 120 s makes the
 * dependent call fail with IA_ECOMM. */
int ia_pipeline_depend(ia_ctx *ctx, ia_ctx *prev, int prev_gen);
int ia_pipeline_generation(ia_ctx *ctx);

/* ---- FLANN-compatible exact index (algorithms.py:56,69,74) -------------------------------- */
/* build_index(pts): pts is n x d fp64 (row-major), d <= 167. */
int ia_index_build(ia_ctx *ctx, const double *pts, int64_t n, int d, ia_index **out);
/* nn_index(q, 1): exact 1-NN, squared L2 in fp64 with numpy's pairwise summation order,
 * lowest index on ties.  q is nq x d fp64; idx_out (nq) int64, dist_out (nq) fp64 (may be NULL). */
int ia_index_query(ia_index *index, const double *q, int64_t nq, int64_t *idx_out, double *dist_out);
void ia_index_destroy(ia_index *index);
/* best_coherence_match (algorithms.py:92-130) for nq B' pixels against the index's rows (the
 * As of create_index, algorithms.py:63-67), one call per batch instead of one per pixel.
 * q: nq x d fp64 query features (BBp_feat); px: nq x 2 int32 (row, col) of each pixel in the
 * B' level of width bp_w; s (n_s x 2 int32) / im (n_s) the raster-order source map of that
 * level, which must hold every causal neighbour of every pixel of the batch (s[r], im[r] for
 * the raster-earlier r in rows row-pad..row, cols col-pad..col+pad); a_h, a_w: A's level
 * shape (DB row = Ap_px2ix(p, im, a_h, a_w), img_preprocess.py:104-106); pad = c.pad_lg (2).
 * Out per pixel: p_out (row, col) = s[r*] + px - r*, img_out = im[r*], rstar_out = r*; or
 * (-1, -1), 0, (0, 0) without a candidate.  Candidates are ranked by sqrt of numpy's pairwise
 * sum of squares, first argmin (np.argmin of norm(..., axis=1)).  IA_EINVAL when a neighbour
 * index reaches beyond n_s or a candidate row beyond the index (an IndexError there). */
int ia_coherence_batch(ia_index *index, const double *q, int64_t nq, const int32_t *px,
                       const int32_t *s, const int32_t *im, int64_t n_s, int a_h, int a_w,
                       int bp_w, int pad, int32_t *p_out, int32_t *img_out, int32_t *rstar_out);

/* ---- GPU preprocessing (img_setup, image_analogies.py:17-94) -------------------- */
/* n_reduce steps of skimage 0.18.3 pyramid_reduce (img_preprocess.py:47-63): scipy.ndimage
 * gaussian_filter (sigma 2/3, mode 'reflect', 7 taps: weights7 = scipy's kernel, symmetric;
 * axes 0 and 1, a colour axis unsmoothed) + order-1 resize to ceil(h/2) x ceil(w/2) clipped to
 * the smoothed image's range.  img (h, w, ch) fp64; out = the n_reduce reduced levels, finest
 * first, concatenated.  Bit-identical to ia_amd.img_preprocess.compute_gaussian_pyramid.
 * mem selects host or device memory for img and out; weights7 is ALWAYS a host array (its
 * four distinct taps travel in the kernel arguments). */
int ia_gaussian_pyramid(ia_ctx *ctx, const double *img, int h, int w, int ch, int n_reduce,
                        const double *weights7, double *out, int mem);
/* out[p, i] = sum_j M9[3 i + j] in[p, j] for npx pixels of 3 channels, in numpy's
 * einsum('ij,klj->kli') order (m0 x0 + m2 x2) + m1 x1 (convert_to_YIQ / convert_to_RGB,
 * img_preprocess.py:6-22).  mem selects host or device memory for in and out; M9 is ALWAYS a
 * host array (copied to the device per call). */
int ia_color_matrix(ia_ctx *ctx, const double *in, int64_t npx, const double *M9, double *out,
                    int mem);

/* ---- kernel tuning ------------------------------------------------------------------------- */
/* Time the split-f16 distance scan (K3h, current "k3_variant") alone: n_rows random DB rows
 * (1 channel), M <= 352 random queries, `reps` back-to-back launches on the context's stream;
 * *us_per_launch = mean device time per launch (HIP events). */
int ia_k3_microbench(ia_ctx *ctx, int64_t n_rows, int M, int reps, double *us_per_launch);

/* ---- host-side helpers (no GPU needed) ---------------------------------------------------- */
/* Merge per-rank candidate winners (dist fp64, global row) into the global winner per query:
 * smallest distance, then smallest row.  cand is world x nq (dist, row) pairs, rank-major. */
int ia_merge_winners(const double *dist, const int64_t *row, int world, int64_t nq,
                     double *dist_out, int64_t *row_out);
/* Budget of handoff-chained waves (fused merge + gather launches whose waves wait for the row
 * above) a context may have in flight deadlock-free: 2 x the resident waves of its n_cu CUs, less
 * 1/16, from the compiled kernel's VGPRs per lane, the occupancy API's workgroups per CU and its
 * workgroup size; 0 = never chain.  ia_init computes it from k_merge_gather itself. */
int ia_chain_budget(int n_cu, int vgprs, int api_blocks_per_cu, int wg_threads);
/* Wavefront schedule of a level (t = col + 3*row): number of steps and max queries per step. */
int ia_wavefront_shape(int h, int w, int64_t *steps, int64_t *max_queries);
/* Pixels of step t: rows r0 .. r0+M-1, pixel (r, t - 3r).  Used by the level driver. */
int ia_wavefront_step(int h, int w, int64_t t, int *r0, int *M);
/* DB tiles [tile0, tile1) owned by `rank` of `world` for a level of n_rows DB rows.  The DB is
 * stored in NT = ceil(n_rows/32) tiles of 32 positions; position j of tile t holds row
 * j*NT + (t * (2654435761 mod NT) mod NT) (tile-strided and tile-scattered, so neighbouring A
 * pixels sit in far-apart tiles).  Tiles are split contiguously over ranks; levels under
 * 64*world tiles are not sharded (every rank owns every tile). */
int ia_shard_tiles(int64_t n_rows, int world, int rank, int64_t *tile0, int64_t *tile1);
/* Pruned levels (certified pruned scan) shard differently: every rank holds the whole
 * Morton-sorted DB, stored shard by shard; shard r = Morton tiles r, r + world, r + 2 world, ...
 * (each covers the whole feature space: balanced pruned work), stored as storage tiles
 * [tile0, tile1).  ia_shard_morton_tile gives the Morton tile of a storage tile. */
int ia_shard_tiles_pruned(int64_t n_rows, int world, int rank, int64_t *tile0, int64_t *tile1);
int64_t ia_shard_morton_tile(int64_t storage_tile, int64_t n_tiles, int world);

#ifdef __cplusplus
}
#endif
#endif /* IA_H_ */
