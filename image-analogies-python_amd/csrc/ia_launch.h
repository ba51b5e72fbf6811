// ia_launch.h — host launchers of the kernels in ia_kernels.hip (used by ia_capi.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include "ia_internal.h"

void ia_launch_means(int ch, const Imgs &A, int n_ap, double *mu, hipStream_t st);
void ia_launch_db_build(const LevelGeo &g, const Imgs &A, const double *mu, float4 *db, unsigned *Rbits, hipStream_t st);
void ia_launch_gather(const LevelGeo &g, const StepDesc &sd, const Imgs &B, const JobSet &jobs, const double *mu, double *q64,
                      double *qn2, float *qf, hipStream_t st);
int ia_k3_qtmax(int KH);
void ia_launch_k3(int KH, int qt, const float4 *db, const float4 *qf, int n_tiles, int tpw, int qt0, int M, int nwg,
                  int row0, int NT, float4 *rec, float *recT, hipStream_t st);
void ia_launch_merge(const LevelGeo &g, const StepDesc &sd, const Imgs &A, const MergeArgs &ma, Winner *win,
                     const JobSet &jobs, bool fused, hipStream_t st);
// fused K4 of step sd + the gather of step nx.sn (K2p when pruned, else K2h; 1-channel levels,
// <= 256 records per query)
void ia_launch_merge_gather(const LevelGeo &g, const StepDesc &sd, const Imgs &A, const MergeArgs &ma, const JobSet &jobs,
                            const Imgs &B, const NextStep &nx, bool pruned, hipStream_t st);
void ia_launch_finish(const LevelGeo &g, const StepDesc &sd, const Imgs &A, const double *db64, const double *q64,
                      const Winner *allwin, int world, int Mstride, const JobSet &jobs, hipStream_t st);
void ia_launch_db64_build(const LevelGeo &g, const Imgs &A, double *db64, hipStream_t st);
int ia_db64_stride(int ch);
void ia_launch_reduce_stats(const unsigned *pstat, int64_t n, unsigned long long *counters, hipStream_t st);
// option "stamps": per launch (min start, max end) ticks over its stride workgroup slots
void ia_launch_stamp_durations(const unsigned long long *stamps, int n, int stride, unsigned long long *span, hipStream_t st,
                               unsigned long long *span2 = nullptr);
void ia_launch_dense_db(int KH, const double *pts, int64_t n, int d, int n_tiles, const double *mu, float4 *db,
                        unsigned *Rbits, hipStream_t st);
void ia_launch_dense_query(int KH, const double *q, int64_t nq, int d, int Mpad, const double *mu, double *qn2, float *qf,
                           hipStream_t st);
void ia_launch_merge_dense(const MergeArgs &ma, const double *pts, int d, const double *q, int64_t nq, int64_t *idx,
                           double *dist, hipStream_t st);
void ia_launch_coherence_batch(const double *pts, int64_t n, int d, const double *q, int64_t nq, const int32_t *px,
                               const int32_t *s, const int32_t *im, int64_t n_s, int a_h, int a_w, int bp_w, int pad,
                               int32_t *p_out, int32_t *img_out, int32_t *r_out, unsigned *err, hipStream_t st);
// split-f16 matcher (IA_MATCH_F16X3)
int ia_ks_for(int ch);
double ia_k3h_tile_bytes(int KS);  // HBM bytes of one split-f16 DB tile (TileFmt)
int ia_k3h_qtmax(int KS);
size_t ia_k3h_lds(int KS, int qt);
void ia_launch_absmax(const double *const *p, const int64_t *n, unsigned *out, hipStream_t st);
void ia_launch_db_build_h(const LevelGeo &g, const Imgs &A, const double *db64, const double *mu, void *db, unsigned *Rbits,
                          hipStream_t st);
void ia_launch_gather_h(const LevelGeo &g, const StepDesc &sd, const Imgs &B, const JobSet &jobs, const double *mu,
                        double *q64, double *qn2, void *qf, hipStream_t st);
void ia_launch_k3h(int KS, int qt, const void *db, const void *qf, int n_tiles, int tpw, int qt0, int M, int nwg, int row0,
                   int NT, float4 *rec, float *recT, int variant, hipStream_t st);
void ia_launch_fill_random_f16(void *p, int64_t n, unsigned seed, hipStream_t st);
// certified pruned scan: per-level setup (ia_prune.hip)
void ia_launch_cov(const double *db64, int64_t NA, int64_t stride, int nwg, const double *mu_part, double *part,
                   double *cov, hipStream_t st);
void ia_launch_proj_keys(const double *db64, int64_t NA, const double *mu_part, const double *basis, double *proj,
                         unsigned *keys, int *rows, float *rnorm, hipStream_t st);
size_t ia_sort_temp_bytes(int64_t n);
int ia_sort_pairs(void *temp, size_t temp_bytes, const unsigned *keys_in, unsigned *keys_out, const int *vals_in,
                  int *vals_out, int64_t n, hipStream_t st);
void ia_launch_table_boxes(const int *sorted_rows, const double *proj, int64_t NA, int n_tiles, int W, int G, int *pos2row,
                           float *boxes, const float *rnorm, float *tnorm, hipStream_t st);
void ia_launch_gather_p(const LevelGeo &g, const StepDesc &sd, const Imgs &B, const JobSet &jobs, const double *mu,
                        double *q64, double *qn2, void *qf, const double *db64, const double *basis, double ufac,
                        float4 *qinfo, const Imgs &A, int img_rows, hipStream_t st, const XOPub *xp = nullptr);
void ia_launch_query_sort(const float4 *qinfo, const void *qf, int Mpad, int KS, int *order, float4 *sq, void *qfs,
                          float4 *tbox, hipStream_t st);
// owner-computes sharded step (exchange = 2): the owner's queries sorted into every rank's area
void ia_launch_query_sort_xo(const float4 *qinfo, const void *qf, const XOSort &xs, hipStream_t st);
size_t ia_k3p_lds(int qt, int Mpad);
void ia_merge_gather_occupancy(int *vgprs, int *blocks_per_cu, int *wg_threads);
// returns IA_EINVAL (nothing launched) when no kernel instance exists for the variant
int ia_launch_k3p(int qt, const void *db, const void *qf, const float4 *qinfo, const float4 *boxes, const int *pos2row,
                   int NT, int qt0, int M, int Mpad, int nwg, float4 *rec, float *recT, unsigned long long *pairs,
                   unsigned long long *tiles, int variant, int step, const int *ord_in, int n_in, int r0, int *ord_out,
                   const float4 *tbox, const float *tnorm, hipStream_t st, int nqb = 1, int qt_end = 0,
                   const XOScan *xo = nullptr, unsigned long long *stamp = nullptr, int rec_wt = 0);
// GPU preprocessing (ia_pyramid.hip)
void ia_launch_pyramid_reduce(const double *in, double *out, double *tmp, double *sm, double *mm, int h, int w, int ch,
                              const double *w7, hipStream_t st);
void ia_launch_color3(const double *in, double *out, int64_t npx, const double *M, hipStream_t st);
// sharded level, peer-write winner exchange (option "exchange" = 1): shard winner -> every rank's
// buffer; fin: wait for the W winners of each query and finish the pixel
void ia_launch_merge_xchg(const LevelGeo &g, const StepDesc &sd, const Imgs &A, const MergeArgs &ma, const XchgArgs &xa,
                          const JobSet &jobs, bool fin, hipStream_t st);
