// ia_capi.cpp — host runtime of libia.so: context, device memory, the per-level skewed
// wavefront scheduler, the FLANN-compatible exact index and the RCCL shard exchange.
// Entry points are declared (with the reference interfaces they replace) in include/ia.h.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ia.h"
#include "ia_internal.h"
#include "ia_launch.h"

#if IA_PROBE & 16
void ia_k3p_probe_dump();
#endif

namespace {

thread_local std::string g_last_error;

// Waves of the handoff-chained launches (k_merge_gather: a gather waits for the merge of the row
// above) of every level in flight in this process.  A wave waits only for its row predecessor
// and no two waves share one, so a stall needs every resident slot held by a waiter whose
// predecessor is not yet dispatched: >= 2 x the resident slots chained waves in flight at once.
// The resident slots come from the compiled k_merge_gather instances (ia_chain_budget, at
// ia_init: VGPRs and the occupancy API; 4 waves per CU at round 4's 264 VGPRs).  A level
// chains only if its widest launch fits in the budget left (ia_synthesize_levels is
// synchronous: its launches are done when it returns); otherwise it runs the separate gather /
// merge launches.  (cfg5's 16-job batches of 512^2 steps, 2,736 waves per launch on three
// streams, hit the 20 s handoff timeout without this.)
static std::atomic<int> g_chain_waves{0};
struct ChainReservation {
  int n = 0;
  ~ChainReservation() {
    if (n) g_chain_waves.fetch_sub(n);
  }
  bool take(int w, int budget) {
    int cur = g_chain_waves.load();
    while (cur + w <= budget)
      if (g_chain_waves.compare_exchange_weak(cur, cur + w)) {
        n = w;
        return true;
      }
    return false;
  }
};

int fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      return fail(IA_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));                 \
  } while (0)
#define NCCL_TRY(expr)                                                                         \
  do {                                                                                         \
    ncclResult_t r_ = (expr);                                                                  \
    if (r_ != ncclSuccess) return fail(IA_ECOMM, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
  } while (0)

// grow-only device buffer
struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return IA_OK;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 256);
    if (hipMalloc(&p, want) != hipSuccess) return fail(IA_ENOMEM, "hipMalloc of " + std::to_string(want) + " bytes failed");
    cap = want;
    return IA_OK;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T *as() const {
    return reinterpret_cast<T *>(p);
  }
};

struct JobBufs {
  DevBuf B, Bc, Bpc, Bp, S, IM, W, DSRC, DDIST, pstat, NN;
  void release() {
    for (DevBuf *b : {&B, &Bc, &Bpc, &Bp, &S, &IM, &W, &DSRC, &DDIST, &pstat, &NN}) b->release();
  }
};

int kh_for(int d_plus_norm) {  // smallest instantiated K3 width that holds d + norm column
  if (d_plus_norm <= 56) return 28;
  if (d_plus_norm <= 112) return 56;
  if (d_plus_norm <= 168) return 84;
  return -1;
}

}  // namespace

struct ia_ctx {
  int dev = 0;
  hipStream_t st = nullptr;
  // uploads (IA_MEM_HOST) and per-level scratch
  DevBuf A, Ac, Ap, Apc;
  std::vector<JobBufs> jb;  // per job of a batch: B-side uploads / outputs, stats words
  DevBuf jobs;              // device JobPtrs[n_jobs]
  DevBuf db, db64, mu, Rbits, q64, qn2, qf, rec, recT, win, allwin, counters, absmax;
  // certified pruned scan (option "prune"): per-level basis, sorted DB table, tile boxes
  DevBuf pr_part, pr_cov, pr_basis, pr_proj, pr_keys, pr_rows, pr_tmp, pos2row, boxes, qinfo, pairs, ord;
  DevBuf qs_order, qs_info, qs_frag, qs_tbox;
  DevBuf tnorm;  // per DB tile of a pruned level: R_t >= max |a'| over its rows (k3p_variant 14/15)  // presorted queries of a step (k3p_variant 11, K2s)
  DevBuf py_in, py_tmp, py_sm, py_mm, py_out;  // GPU preprocessing (ia_gaussian_pyramid, ia_color_matrix)
  std::vector<double> basis_h;   // staging of the basis upload (lives until the copy ran)
  int64_t prune_min_rows = IA_PRUNE_MIN_ROWS;  // option "prune_min_rows": smallest DB that prunes
  int prune = 1;
  int row_source = 0;            // option "row_source": exact rows from 0 = the fp64 row DB, 1 = the A images
  int shard_emulate = 1;         // option "shard_emulate": W > 1 runs a W-way DB shard on this device
  int shard_unpruned = 0;        // option "shard_unpruned": 1 = shard levels that scan unpruned too
  int prune_group = 1;           // option "prune_group": Morton tiles interleaved in groups of G (ia_prune.hip k_make_table)
  int matcher = IA_MATCH_F16X3;  // option "matcher"
  int k3p_variant = 24;          // option "k3p_variant": pruned-scan kernel version (ia_k3h.hip k3h_prune*)
  int k3_variant = 1;            // option "k3_variant": K3h epilogue (0 compare/select, 1 packed index)
  int k3p_blocks = 1;            // option "k3p_blocks": 1 = a wide step's presorted pruned scan is one launch over
                                 // all its query blocks (2-D grid); 0 = one launch per block
  int fuse_gather = 1;           // option "fuse_gather": 1 = K4 of step t and K2p of step t + 1 in one launch
  int fuse_unpruned = 0;         // option "fuse_unpruned": 1 = also on unpruned levels (K4 + K2h)
  HandSlot *hand = nullptr;      // its per-row handoff slots (uncached)
  int hand_rows = 0;
  int prefetch_next = 1;         // option "prefetch_next" (NextStep::prefetch)
  int early_gather = 1;          // option "early_gather" (NextStep::early)
  int nn_bound = 1;              // option "nn_bound" (JobPtrs::nn): the pruned one-rank levels' gathers also
                                 // bound U' by the causal neighbours' exact NN rows, shifted
  int fuse_sort = 0;             // option "fuse_sort": the fused gathers of step t + 1 also sort it (NextStep::kslot);
                                 // 2 = on levels whose widest step has >= IA_FUSE_SORT_MINQ queries; off by
                                 // default: no gain left with nn_bound
  int chain_budget = 0;          // waves of handoff-chained launches this context's CUs hold deadlock-free
  int scan_wgs = IA_NWG_H;       // option "scan_wgs": workgroups of a pruned scan launch (<= one per CU)
                                 // (ia_init: 2 x the resident merge-gather waves - a margin; see g_chain_waves)
  unsigned long long *kslot = nullptr;  // their per-query key slots (uncached)
  int kslot_n = 0;
  unsigned hseq = 0;
  // per-step K3 timing (optional)
  int time_dist = 0;
  int stamps = 0;                 // option "stamps": per-launch device time from kernel stamps
  int rec_wt = 1;                 // option "rec_wt": K3p records stored write-through
  DevBuf stamp_k3, stamp_mg, stamp_dur;
  std::vector<hipEvent_t> evs, evg, evm;  // sampled steps: K3, K2 and K4 brackets
  hipEvent_t lv0 = nullptr, lv1 = nullptr, lv2 = nullptr;
  hipEvent_t kb[4] = {nullptr, nullptr, nullptr, nullptr};  // per level: K1b start / end, K1 start / end
  // multi-GPU
  int rank = 0, world = 1;
  ncclComm_t comm = nullptr;
  int exchange = 0;               // option "exchange": 0 = RCCL all-gather + finish, 1 = peer-write merge,
                                  // 2 = owner-computes (rank o owns job o; every rank scans its shard for all)
  DevBuf xo_inv;                  // exchange = 2: the owners' query -> slot tables of the current step
  int xo_presort = 0;             // option "xo_presort": 1 = owners always sort with K2s (tests)
  int xo_wait = 0;                // option "xo_wait": 1 = the fused merge waits for every owner's next
                                  // queries (one wave), so the next scan does not spin on all CUs
  void *xbuf = nullptr;           // this process's exchange buffer (uncached, IPC-exportable)
  int xbuf_w = 0;                 // ranks the buffer was sized for
  XSlot *xpeer[IA_XCHG_MAXW] = {};  // every rank's buffer in this address space (ia_xchg_open)
  bool xmapped[IA_XCHG_MAXW] = {};  // opened through hipIpcOpenMemHandle (closed on destroy)
  unsigned xseq = 0;              // exchange sequence number (one per sharded step, same on every rank)
  bool xfresh = false;            // the buffer was zeroed by ia_xchg_alloc and not opened since
  DevBuf xerr;
  // level pipelining: a recording context publishes, per level call (a
  // generation), the wavefront steps it has enqueued, each followed by an event; a context told
  // to depend on it (ia_pipeline_depend) makes each of its steps wait for the steps of that
  // generation it reads from (level l + 1 step t reads B' of level l steps <= t / 2 + 4)
  int p_record = 0;                          // option "pipeline_record"
  int p_last = 0;                            // option "pipeline_last": the next level call has no
                                             // dependents (no per-step events; one call only)
  std::vector<hipEvent_t> p_ev[3];           // per generation mod 3: one event per step
  std::atomic<long long> p_enq{-1};          // last step of the current generation enqueued
  std::atomic<long long> p_T{0};             // steps of the current generation
  std::atomic<int> p_gen{0}, p_done{0};      // current / last finished generation
  ia_ctx *dep = nullptr;                     // the next level call waits on dep's generation dep_gen
  int dep_gen = 0;
};

struct ia_index {
  ia_ctx *ctx = nullptr;
  int64_t n = 0;
  int d = 0, KH = 0, n_tiles = 0, tpw = 0, nwg = 0;
  DevBuf pts, db, mu, Rbits, q, q64, qn2, qf, rec, recT, idx, dist, counters;
  DevBuf cpx, cs, cim, cout;  // ia_coherence_batch staging
};

namespace {

// cyclic Jacobi eigen-decomposition of a symmetric n x n matrix (row-major, overwritten);
// V's column k is the eigenvector of eigenvalue w[k]
void jacobi_eig(int n, std::vector<double> &A, std::vector<double> &V, std::vector<double> &w) {
  V.assign((size_t)n * n, 0.);
  for (int i = 0; i < n; i++) V[(size_t)i * n + i] = 1.;
  auto a = [&](int i, int j) -> double & { return A[(size_t)i * n + j]; };
  for (int sweep = 0; sweep < 100; sweep++) {
    double off = 0., dia = 0.;
    for (int p = 0; p < n; p++) {
      dia += a(p, p) * a(p, p);
      for (int q = p + 1; q < n; q++) off += a(p, q) * a(p, q);
    }
    if (off <= 1e-32 * dia || off == 0.) break;
    for (int p = 0; p < n - 1; p++) {
      for (int q = p + 1; q < n; q++) {
        const double apq = a(p, q);
        if (apq == 0.) continue;
        const double theta = (a(q, q) - a(p, p)) / (2. * apq);
        const double t = (theta >= 0. ? 1. : -1.) / (std::fabs(theta) + std::sqrt(theta * theta + 1.));
        const double cs = 1. / std::sqrt(t * t + 1.), sn = t * cs;
        for (int k = 0; k < n; k++) {  // columns p, q
          const double akp = a(k, p), akq = a(k, q);
          a(k, p) = cs * akp - sn * akq;
          a(k, q) = sn * akp + cs * akq;
        }
        for (int k = 0; k < n; k++) {  // rows p, q
          const double apk = a(p, k), aqk = a(q, k);
          a(p, k) = cs * apk - sn * aqk;
          a(q, k) = sn * apk + cs * aqk;
        }
        for (int k = 0; k < n; k++) {
          const double vkp = V[(size_t)k * n + p], vkq = V[(size_t)k * n + q];
          V[(size_t)k * n + p] = cs * vkp - sn * vkq;
          V[(size_t)k * n + q] = sn * vkp + cs * vkq;
        }
      }
    }
  }
  w.resize(n);
  for (int i = 0; i < n; i++) w[i] = a(i, i);
}

// Per-level setup of the certified pruned scan (ia_prune.hip): covariance of
// the centred fp64 DB (sampled) -> top IA_NPC eigenvectors (host Jacobi) -> projections and
// Morton keys of every row -> radix sort -> position -> row table + per-tile projection boxes.
// Sets g.pos2row; *ufac = the U' factor of ia_prune.h.  One host sync (the covariance).
int prepare_prune(ia_ctx *c, LevelGeo &g, const double *mu, int W, double *ufac) {
  constexpr int D = 55, NPAIR = D * (D + 1) / 2, NWG_COV = 256;
  const int64_t NA = g.NA, NT = g.n_tiles;
  const int64_t stride = std::max<int64_t>(1, NA / 65536), nsamp = (NA + stride - 1) / stride;
  int rc;
  if ((rc = c->pr_part.ensure((size_t)NWG_COV * NPAIR * 8)) || (rc = c->pr_cov.ensure((size_t)NPAIR * 8)) ||
      (rc = c->pr_basis.ensure((size_t)(IA_NPC * D + IA_NPC) * 8)) || (rc = c->pr_proj.ensure((size_t)NA * (IA_NPC * 8 + 4))) ||
      (rc = c->pr_keys.ensure((size_t)NA * 8)) || (rc = c->pr_rows.ensure((size_t)NA * 8)) ||
      (rc = c->pos2row.ensure((size_t)NT * IA_TILE * 4)) || (rc = c->boxes.ensure((size_t)NT * 2 * IA_NPC * 4)) ||
      (rc = c->tnorm.ensure((size_t)NT * 4)))
    return rc;
  const size_t sort_bytes = ia_sort_temp_bytes(NA);
  if ((rc = c->pr_tmp.ensure(sort_bytes))) return rc;
  ia_launch_cov(c->db64.as<double>(), NA, stride, NWG_COV, mu, c->pr_part.as<double>(), c->pr_cov.as<double>(), c->st);
  std::vector<double> cov(NPAIR);
  HIP_TRY(hipMemcpyAsync(cov.data(), c->pr_cov.p, NPAIR * 8, hipMemcpyDeviceToHost, c->st));
  HIP_TRY(hipStreamSynchronize(c->st));
  std::vector<double> A((size_t)D * D), V, w;
  for (int f = 0, p = 0; f < D; f++)
    for (int h = f; h < D; h++, p++) A[(size_t)f * D + h] = A[(size_t)h * D + f] = cov[p] / (double)nsamp;
  jacobi_eig(D, A, V, w);
  std::vector<int> idx(D);
  for (int i = 0; i < D; i++) idx[i] = i;
  std::stable_sort(idx.begin(), idx.end(), [&](int x, int y) { return w[x] > w[y]; });
  c->basis_h.assign((size_t)IA_NPC * D + IA_NPC, 0.);
  for (int i = 0; i < IA_NPC; i++) {
    double nrm = 0.;
    for (int f = 0; f < D; f++) nrm += V[(size_t)f * D + idx[i]] * V[(size_t)f * D + idx[i]];
    nrm = std::sqrt(nrm);
    for (int f = 0; f < D; f++) c->basis_h[(size_t)i * D + f] = V[(size_t)f * D + idx[i]] / nrm;
    const double lam = w[idx[i]];
    c->basis_h[(size_t)IA_NPC * D + i] = lam > 0. ? 1. / (4. * std::sqrt(lam)) : 0.;
  }
  // deviation of the basis from orthonormality: lambda_max(U^T U) <= 1 + sum |G - I|
  long double delta = 0.L;
  for (int i = 0; i < IA_NPC; i++)
    for (int j = 0; j < IA_NPC; j++) {
      long double gij = 0.L;
      for (int f = 0; f < D; f++) gij += (long double)c->basis_h[(size_t)i * D + f] * c->basis_h[(size_t)j * D + f];
      delta += std::fabs((double)(gij - (i == j ? 1.L : 0.L)));
    }
  *ufac = (1.0 + 2.0 * (double)delta + 1e-15) * (1.0 + std::ldexp(1.0, -17)) * (1.0 + std::ldexp(1.0, -19));
  HIP_TRY(hipMemcpyAsync(c->pr_basis.p, c->basis_h.data(), c->basis_h.size() * 8, hipMemcpyHostToDevice, c->st));
  unsigned *keys = c->pr_keys.as<unsigned>();
  int *rows = c->pr_rows.as<int>();
  float *rnorm = reinterpret_cast<float *>(c->pr_proj.as<double>() + NA * IA_NPC);  // |a'| per row, rounded up
  ia_launch_proj_keys(c->db64.as<double>(), NA, mu, c->pr_basis.as<double>(), c->pr_proj.as<double>(), keys, rows, rnorm,
                      c->st);
  if (ia_sort_pairs(c->pr_tmp.p, sort_bytes, keys, keys + NA, rows, rows + NA, NA, c->st) != 0)
    return fail(IA_EHIP, "prepare_prune: radix sort failed");
  ia_launch_table_boxes(rows + NA, c->pr_proj.as<double>(), NA, (int)NT, W, c->prune_group, c->pos2row.as<int>(),
                        c->boxes.as<float>(), rnorm,
                        c->tnorm.as<float>(), c->st);
  HIP_TRY(hipGetLastError());
  g.pos2row = c->pos2row.as<int>();
  return IA_OK;
}

}  // namespace

extern "C" {

const char *ia_last_error(void) { return g_last_error.c_str(); }
int ia_version(void) { return 1; }

int ia_init(int device, ia_ctx **out) {
  if (!out) return fail(IA_EINVAL, "ia_init: out is NULL");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(IA_ENODEV, "ia_init: no HIP device visible");
  if (device < 0 || device >= n) return fail(IA_EINVAL, "ia_init: device index out of range");
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(IA_ENODEV, std::string("ia_init: libia is built for gfx950 only, device is ") + prop.gcnArchName);
  HIP_TRY(hipSetDevice(device));
  ia_ctx *c = new ia_ctx();
  c->dev = device;
  // IA_CU_SPLIT=k/n (rehearsals of the multi-rank exchanges with n ranks sharing ONE GPU only):
  // this context's stream runs on CU slice k of n, so a rank's kernel that waits for a peer's
  // progress never holds the CUs the peer's kernels need (on separate GPUs nothing is shared)
  int split_k = 0, split_n = 0;
  if (const char *e = std::getenv("IA_CU_SPLIT")) {
    if (std::sscanf(e, "%d/%d", &split_k, &split_n) != 2 || split_n < 1 || split_k < 0 || split_k >= split_n) split_n = 0;
  }
  hipError_t se;
  if (split_n > 1) {
    const int ncu = prop.multiProcessorCount;
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    for (int cu = ncu * split_k / split_n; cu < ncu * (split_k + 1) / split_n; cu++) mask[cu / 32] |= 1u << (cu % 32);
    se = hipExtStreamCreateWithCUMask(&c->st, (uint32_t)mask.size(), mask.data());
  } else {
    se = hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking);
  }
  if (se != hipSuccess) {
    delete c;
    return fail(IA_EHIP, "ia_init: hipStreamCreate failed");
  }
  {  // g_chain_waves: the resident k_merge_gather waves of this context's CU slice, twice, less 1/16
    const int ncu = split_n > 1 ? prop.multiProcessorCount / split_n : prop.multiProcessorCount;
    int vg = 0, nb = 0, wt = 0;
    ia_merge_gather_occupancy(&vg, &nb, &wt);
    c->chain_budget = ia_chain_budget(ncu, vg, nb, wt);  // 0: never chain (separate launches)
  }
  hipEventCreate(&c->lv0);
  hipEventCreate(&c->lv1);
  hipEventCreate(&c->lv2);
  for (hipEvent_t &e : c->kb) hipEventCreate(&e);
  *out = c;
  return IA_OK;
}

void ia_destroy(ia_ctx *c) {
  if (!c) return;
  hipSetDevice(c->dev);
  hipStreamSynchronize(c->st);
  for (JobBufs &b : c->jb) b.release();
  for (DevBuf *b : {&c->A, &c->Ac, &c->Ap, &c->Apc, &c->jobs, &c->db, &c->db64,
                    &c->mu, &c->Rbits, &c->q64, &c->qn2, &c->qf, &c->rec, &c->recT, &c->win, &c->allwin, &c->counters, &c->absmax,
                    &c->pr_part, &c->pr_cov, &c->pr_basis, &c->pr_proj, &c->pr_keys, &c->pr_rows, &c->pr_tmp, &c->pos2row,
                    &c->boxes, &c->qinfo, &c->pairs, &c->ord, &c->qs_order, &c->qs_info, &c->qs_frag, &c->qs_tbox, &c->tnorm,
                    &c->stamp_k3, &c->stamp_mg, &c->stamp_dur,
                    &c->py_in, &c->py_tmp, &c->py_sm, &c->py_mm, &c->py_out})
    b->release();
  for (auto *v : {&c->evs, &c->evg, &c->evm, &c->p_ev[0], &c->p_ev[1], &c->p_ev[2]})
    for (hipEvent_t e : *v) hipEventDestroy(e);
  for (hipEvent_t e : c->kb) hipEventDestroy(e);
  hipEventDestroy(c->lv0);
  hipEventDestroy(c->lv1);
  hipEventDestroy(c->lv2);
  if (c->comm) ncclCommDestroy(c->comm);
  for (int p = 0; p < IA_XCHG_MAXW; p++)
    if (c->xmapped[p]) hipIpcCloseMemHandle(c->xpeer[p]);
  if (c->xbuf) hipFree(c->xbuf);
  if (c->hand) hipFree(c->hand);
  if (c->kslot) hipFree(c->kslot);
  c->xerr.release();
  c->xo_inv.release();
  hipStreamDestroy(c->st);
  delete c;
}

int ia_set_option(ia_ctx *c, const char *name, int value) {
  if (!c || !name) return fail(IA_EINVAL, "ia_set_option: NULL argument");
  if (!std::strcmp(name, "time_dist")) {
    c->time_dist = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "rec_wt")) {
    if (value != 0 && value != 1) return fail(IA_EINVAL, "ia_set_option: rec_wt must be 0 or 1");
    c->rec_wt = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "stamps")) {
    if (value != 0 && value != 1) return fail(IA_EINVAL, "ia_set_option: stamps must be 0 or 1");
    c->stamps = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "k3p_variant")) {  // 24 / 25 two passes (a hi stream three
                                            // tiles deep, then the passing tiles' chains); 22 hi-only
                                            // stream with the chains one tile later; 20 / 21 whole tiles,
                                            // corrections fused on query-tile pairs.  In-kernel sort up to
                                            // 512 queries (20, 22, 24), presorted above (21, 25); the other
                                            // versions are in git history
    if (value != 20 && value != 21 && value != 22 && value != 24 && value != 25)
      return fail(IA_EINVAL, "ia_set_option: k3p_variant is 20, 21, 22, 24 or 25");
    c->k3p_variant = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "k3_variant")) {
    if (value != 1) return fail(IA_EINVAL, "ia_set_option: k3_variant is 1 (the packed-index epilogue; the others are in git history)");
    return IA_OK;
  }
  if (!std::strcmp(name, "prune_group")) {
    if (value != 1 && value != 2 && value != 4 && value != 8)
      return fail(IA_EINVAL, "ia_set_option: prune_group must be 1, 2, 4 or 8");
    c->prune_group = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "prune_min_rows")) {
    if (value < 1) return fail(IA_EINVAL, "ia_set_option: prune_min_rows must be >= 1");
    c->prune_min_rows = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "row_source")) {
    if (value != 0) return fail(IA_EINVAL, "ia_set_option: row_source is 0 (the image-gathered rows, measured slower, are in git history only)");
    c->row_source = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "shard_emulate")) {
    if (value < 1 || value > 64) return fail(IA_EINVAL, "ia_set_option: shard_emulate must be 1..64");
    c->shard_emulate = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "prune")) {
    if (value != 0 && value != 1) return fail(IA_EINVAL, "ia_set_option: prune must be 0 or 1");
    c->prune = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "shard_unpruned")) {
    if (value != 0 && value != 1) return fail(IA_EINVAL, "ia_set_option: shard_unpruned must be 0 or 1");
    c->shard_unpruned = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "k3p_blocks")) {
    if (value != 0 && value != 1) return fail(IA_EINVAL, "ia_set_option: k3p_blocks must be 0 or 1");
    c->k3p_blocks = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "fuse_gather")) {
    if (value != 0 && value != 1) return fail(IA_EINVAL, "ia_set_option: fuse_gather must be 0 or 1");
    c->fuse_gather = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "nn_bound")) {
    if (value != 0 && value != 1) return fail(IA_EINVAL, "ia_set_option: nn_bound must be 0 or 1");
    c->nn_bound = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "early_gather")) {
    if (value != 0 && value != 1) return fail(IA_EINVAL, "ia_set_option: early_gather must be 0 or 1");
    c->early_gather = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "prefetch_next")) {
    if (value != 0 && value != 1) return fail(IA_EINVAL, "ia_set_option: prefetch_next must be 0 or 1");
    c->prefetch_next = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "fuse_sort")) {
    if (value < 0 || value > 2) return fail(IA_EINVAL, "ia_set_option: fuse_sort must be 0, 1 or 2");
    c->fuse_sort = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "fuse_unpruned")) {
    if (value != 0 && value != 1) return fail(IA_EINVAL, "ia_set_option: fuse_unpruned must be 0 or 1");
    c->fuse_unpruned = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "pipeline_last")) {
    if (value != 0 && value != 1) return fail(IA_EINVAL, "ia_set_option: pipeline_last must be 0 or 1");
    c->p_last = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "pipeline_record")) {
    if (value != 0 && value != 1) return fail(IA_EINVAL, "ia_set_option: pipeline_record must be 0 or 1");
    c->p_record = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "stream_priority")) {
    // 0 = default, 1 = high, 2 = low: the stream is recreated (idle contexts only); level
    // pipelining gives the finest level's context the high priority so the
    // coarser levels' kernels fill its gaps instead of delaying its steps
    if (value < 0 || value > 2) return fail(IA_EINVAL, "ia_set_option: stream_priority must be 0, 1 (high) or 2 (low)");
    if (std::getenv("IA_CU_SPLIT")) return fail(IA_EINVAL, "ia_set_option: stream_priority with IA_CU_SPLIT");
    HIP_TRY(hipSetDevice(c->dev));
    int least = 0, greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_TRY(hipStreamSynchronize(c->st));
    hipStream_t ns = nullptr;
    HIP_TRY(hipStreamCreateWithPriority(&ns, hipStreamNonBlocking, value == 0 ? 0 : value == 1 ? greatest : least));
    hipStreamDestroy(c->st);
    c->st = ns;
    return IA_OK;
  }
  if (!std::strcmp(name, "scan_wgs")) {
    if (value < 8 || value > IA_NWG_H || value % 8) return fail(IA_EINVAL, "ia_set_option: scan_wgs must be a multiple of 8 in [8, 256]");
    c->scan_wgs = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "xo_wait")) {
    if (value != 0 && value != 1) return fail(IA_EINVAL, "ia_set_option: xo_wait must be 0 or 1");
    c->xo_wait = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "xo_presort")) {
    if (value != 0 && value != 1) return fail(IA_EINVAL, "ia_set_option: xo_presort must be 0 or 1");
    c->xo_presort = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "exchange")) {
    if (value < 0 || value > 2)
      return fail(IA_EINVAL, "ia_set_option: exchange must be 0 (RCCL), 1 (peer-write winners) or 2 (owner computes)");
    c->exchange = value;
    return IA_OK;
  }
  if (!std::strcmp(name, "matcher")) {
    if (value != IA_MATCH_F32 && value != IA_MATCH_F16X3) return fail(IA_EINVAL, "ia_set_option: matcher must be 0 or 1");
    c->matcher = value;
    return IA_OK;
  }
  return fail(IA_EINVAL, std::string("ia_set_option: unknown option ") + name);
}

int ia_comm_unique_id(unsigned char id_out[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  std::memcpy(id_out, &id, 128);
  return IA_OK;
}

int ia_comm_init(ia_ctx *c, int rank, int world, const unsigned char id[128]) {
  if (!c || world < 1 || rank < 0 || rank >= world) return fail(IA_EINVAL, "ia_comm_init: bad rank/world");
  HIP_TRY(hipSetDevice(c->dev));
  if (c->comm) ncclCommDestroy(c->comm);
  c->comm = nullptr;
  // the RCCL all-gather replaces any peer-write exchange opened before (ia_xchg_open)
  for (int p = 0; p < IA_XCHG_MAXW; p++) {
    if (c->xmapped[p]) hipIpcCloseMemHandle(c->xpeer[p]);
    c->xmapped[p] = false;
    c->xpeer[p] = nullptr;
  }
  c->exchange = 0;
  c->rank = rank;
  c->world = world;
  if (world == 1) return IA_OK;
  ncclUniqueId uid;
  std::memcpy(&uid, id, 128);
  NCCL_TRY(ncclCommInitRank(&c->comm, world, uid, rank));
  return IA_OK;
}

// owner o's K2s of an owner-computes step: its queries sorted into every rank's area (area(p))
extern "C++" template <class AreaFn>
static void ia_launch_query_sort_xo_owner(ia_ctx *c, const LevelGeo &g, const float4 *qinfo, const void *qf,
                                          const StepDesc &sd, int owner, int QTs, unsigned seq, int W, AreaFn area) {
  (void)g;
  XOSort xs{};
  xs.inv = c->xo_inv.as<int>();
  xs.W = W;
  for (int p = 0; p < xs.W; p++) xs.area[p] = area(p);
  xs.q0 = 0;
  xs.Mj = sd.M;
  xs.tile0 = owner * QTs;
  xs.QTs = QTs;
  xs.seq = seq;
  ia_launch_query_sort_xo(qinfo, qf, xs, c->st);
}

// fresh = true (ia_xchg_alloc, before the ranks swap handles): a reused buffer is zeroed too and
// the sequence restarts, so no seq word left from an earlier exchange (or an emulated run on this
// context) can match the restarted sequence; the handle swap orders every rank's zeroing before
// any peer's first store
static int xchg_alloc(ia_ctx *c, int world, bool fresh = false) {
  const size_t bytes = ia_xslots_bytes(world) + 2 * XOLayout::PARITY;
  if (c->xbuf && c->xbuf_w >= world) {
    if (fresh) {
      HIP_TRY(hipStreamSynchronize(c->st));
      HIP_TRY(hipMemset(c->xbuf, 0, ia_xslots_bytes(c->xbuf_w) + 2 * XOLayout::PARITY));
      HIP_TRY(hipDeviceSynchronize());
      c->xbuf_w = world;
      c->xseq = 0;
      c->xfresh = true;
    }
    return IA_OK;
  }
  if (c->xbuf) hipFree(c->xbuf);
  c->xbuf = nullptr;
  // winner slots (exchange = 1) + two parities of the owner-computes area (exchange = 2)
  // uncached: peers' xGMI stores and this device's polling loads meet in memory, not in an L2
  HIP_TRY(hipExtMallocWithFlags(&c->xbuf, bytes, hipDeviceMallocUncached));
  HIP_TRY(hipMemset(c->xbuf, 0, bytes));
  HIP_TRY(hipDeviceSynchronize());
  c->xbuf_w = world;
  c->xseq = 0;
  c->xfresh = fresh;
  int rc;
  if ((rc = c->xerr.ensure(4))) return rc;
  return IA_OK;
}

int ia_xchg_alloc(ia_ctx *c, int world, unsigned char handle_out[64]) {
  if (!c || !handle_out || world < 1 || world > IA_XCHG_MAXW) return fail(IA_EINVAL, "ia_xchg_alloc: world must be 1..16");
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "hipIpcMemHandle_t size");
  HIP_TRY(hipSetDevice(c->dev));
  int rc;
  if ((rc = xchg_alloc(c, world, true))) return rc;
  hipIpcMemHandle_t h;
  HIP_TRY(hipIpcGetMemHandle(&h, c->xbuf));
  std::memcpy(handle_out, &h, 64);
  return IA_OK;
}

int ia_xchg_open(ia_ctx *c, int rank, int world, const unsigned char *handles) {
  if (!c || !handles || world < 1 || world > IA_XCHG_MAXW || rank < 0 || rank >= world)
    return fail(IA_EINVAL, "ia_xchg_open: bad rank / world");
  if (!c->xbuf || c->xbuf_w != world || !c->xfresh)
    return fail(IA_EINVAL, "ia_xchg_open: call ia_xchg_alloc with this world first (once per ia_xchg_open)");
  HIP_TRY(hipSetDevice(c->dev));
  for (int p = 0; p < IA_XCHG_MAXW; p++)
    if (c->xmapped[p]) {
      hipIpcCloseMemHandle(c->xpeer[p]);
      c->xmapped[p] = false;
    }
  for (int p = 0; p < world; p++) {
    if (p == rank) {
      c->xpeer[p] = (XSlot *)c->xbuf;
      continue;
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles + (size_t)64 * p, 64);
    void *ptr = nullptr;
    HIP_TRY(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess));
    c->xpeer[p] = (XSlot *)ptr;
    c->xmapped[p] = true;
  }
  if (c->comm) ncclCommDestroy(c->comm);
  c->comm = nullptr;
  c->rank = rank;
  c->world = world;
  if (c->exchange == 0) c->exchange = 1;  // keep 2 (owner computes) when it was chosen before
  c->xseq = 0;  // the buffer was zeroed by ia_xchg_alloc: no stale seq word matches the new sequence
  c->xfresh = false;
  return IA_OK;
}

int ia_pipeline_depend(ia_ctx *c, ia_ctx *prev, int prev_gen) {
  if (!c || (prev && (prev == c || !prev->p_record || prev_gen < 1)))
    return fail(IA_EINVAL, "ia_pipeline_depend: prev must be another context with pipeline_record = 1 and prev_gen >= 1");
  c->dep = prev;
  c->dep_gen = prev ? prev_gen : 0;
  return IA_OK;
}

int ia_pipeline_generation(ia_ctx *c) { return c ? c->p_gen.load() : -1; }

int ia_chain_budget(int n_cu, int vgprs, int api_blocks_per_cu, int wg_threads) {
  // resident waves per CU: the VGPR bound (512 registers per lane and SIMD, allocated in
  // granules of 8, at most 8 waves per SIMD, 4 SIMDs) and the occupancy API's workgroups; above
  // 3 waves per SIMD the SGPR file can bind too, where the API is known to answer one workgroup
  // too many (MI355X_MICROARCH.md, residency): then one workgroup per CU less
  if (n_cu <= 0 || vgprs <= 0 || api_blocks_per_cu <= 0 || wg_threads <= 0) return 0;
  const int alloc = (vgprs + 7) / 8 * 8;
  const int per_simd = alloc > 512 ? 0 : std::min(8, 512 / alloc);
  const int wpb = (wg_threads + IA_WAVE - 1) / IA_WAVE;
  int per_cu = std::min(4 * per_simd, api_blocks_per_cu * wpb);
  if (per_simd > 3) per_cu = std::min(per_cu, (api_blocks_per_cu - 1) * wpb);
  if (per_cu <= 0) return 0;
  const int slots = per_cu * n_cu;
  return 2 * slots - (2 * slots) / 16;
}
int ia_wavefront_shape(int h, int w, int64_t *steps, int64_t *max_queries) {
  if (h < 1 || w < 1) return fail(IA_EINVAL, "ia_wavefront_shape: empty level");
  if (steps) *steps = (int64_t)w + 3 * (int64_t)(h - 1);
  if (max_queries) *max_queries = std::min<int64_t>(h, (w + 2) / 3);
  return IA_OK;
}

int ia_wavefront_step(int h, int w, int64_t t, int *r0, int *M) {
  if (h < 1 || w < 1 || t < 0 || t >= (int64_t)w + 3 * (int64_t)(h - 1)) return fail(IA_EINVAL, "ia_wavefront_step: bad step");
  const int64_t r_lo = std::max<int64_t>(0, (t - w + 1 + 2) / 3);  // ceil((t - w + 1) / 3), t - w + 3 > 0
  const int64_t r_hi = std::min<int64_t>(h - 1, t / 3);
  *r0 = (int)r_lo;
  *M = (int)(r_hi - r_lo + 1);
  return IA_OK;
}

#define IA_FUSE_SORT_MAXW 768  // waves of a k_merge_gather launch whose gathers sort the next step
#define IA_FUSE_SORT_MINQ 512  // fuse_sort 2: the widest step's queries (all jobs) from which the gathers sort

static bool shard_level(int64_t n_tiles, int world) { return world > 1 && n_tiles >= 64 * (int64_t)world; }

int ia_shard_tiles(int64_t n_rows, int world, int rank, int64_t *tile0, int64_t *tile1) {
  if (n_rows < 1 || world < 1 || rank < 0 || rank >= world || !tile0 || !tile1)
    return fail(IA_EINVAL, "ia_shard_tiles: bad args");
  const int64_t n_tiles = (n_rows + IA_TILE - 1) / IA_TILE;
  if (!shard_level(n_tiles, world)) {
    *tile0 = 0;
    *tile1 = n_tiles;
    return IA_OK;
  }
  *tile0 = n_tiles * rank / world;
  *tile1 = n_tiles * (rank + 1) / world;
  return IA_OK;
}

int ia_shard_tiles_pruned(int64_t n_rows, int world, int rank, int64_t *tile0, int64_t *tile1) {
  if (n_rows < 1 || world < 1 || rank < 0 || rank >= world || !tile0 || !tile1)
    return fail(IA_EINVAL, "ia_shard_tiles_pruned: bad args");
  const int64_t n_tiles = (n_rows + IA_TILE - 1) / IA_TILE;
  if (!shard_level(n_tiles, world)) {
    *tile0 = 0;
    *tile1 = n_tiles;
    return IA_OK;
  }
  *tile0 = ia_shard_off(n_tiles, world, rank);
  *tile1 = ia_shard_off(n_tiles, world, rank + 1);
  return IA_OK;
}

int64_t ia_shard_morton_tile(int64_t storage_tile, int64_t n_tiles, int world) {
  if (world < 1 || n_tiles < 1 || storage_tile < 0 || storage_tile >= n_tiles) return -1;
  return world > 1 ? ia_shard_morton_tile_(storage_tile, n_tiles, world) : storage_tile;
}

int ia_merge_winners(const double *dist, const int64_t *row, int world, int64_t nq, double *dist_out,
                     int64_t *row_out) {
  if (!dist || !row || !dist_out || !row_out || world < 1 || nq < 0) return fail(IA_EINVAL, "ia_merge_winners: bad args");
  for (int64_t m = 0; m < nq; m++) {
    double bd = dist[m];
    int64_t bi = row[m];
    for (int k = 1; k < world; k++) {  // identical order on every rank (k_finish_level)
      const double d = dist[(int64_t)k * nq + m];
      const int64_t i = row[(int64_t)k * nq + m];
      if (d < bd || (d == bd && i < bi)) {
        bd = d;
        bi = i;
      }
    }
    dist_out[m] = bd;
    row_out[m] = bi;
  }
  return IA_OK;
}

// ------------------------------------------------------------------------------------------
// fast path: one pyramid level (image_analogies.py:130-239)
// ------------------------------------------------------------------------------------------
static int stage(ia_ctx *c, DevBuf &buf, const void *src, size_t bytes, int mem, const void **dev) {
  if (mem == IA_MEM_DEVICE) {
    *dev = src;
    return IA_OK;
  }
  int rc = buf.ensure(bytes);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(buf.p, src, bytes, hipMemcpyHostToDevice, c->st));
  *dev = buf.p;
  return IA_OK;
}

static int check_level_args(const ia_level_args *a) {
  if (a->ch < 1 || a->ch > 3) return fail(IA_EINVAL, "ia_synthesize_level: ch must be 1, 2 or 3");
  if (a->n_ap < 1 || a->a_h < 1 || a->a_w < 1 || a->b_h < 1 || a->b_w < 1)
    return fail(IA_EINVAL, "ia_synthesize_level: empty image or no A' image");
  if (!a->A || !a->Ac || !a->Ap || !a->Apc || !a->B || !a->Bc || !a->Bpc || !a->Bp || !a->weights || !a->s_out ||
      !a->im_out)
    return fail(IA_EINVAL, "ia_synthesize_level: NULL image pointer");
  if (a->mem != IA_MEM_HOST && a->mem != IA_MEM_DEVICE) return fail(IA_EINVAL, "ia_synthesize_level: bad mem kind");
  if ((a->dbg_src == nullptr) != (a->dbg_dist == nullptr))
    return fail(IA_EINVAL, "ia_synthesize_level: dbg_src and dbg_dist are given together or not at all");
  if ((int64_t)a->n_ap * a->a_h * a->a_w >= (int64_t)INT32_MAX)
    return fail(IA_EINVAL, "ia_synthesize_level: DB rows exceed int32 row ids");
  return IA_OK;
}

int ia_synthesize_level(ia_ctx *c, const ia_level_args *a, ia_stats *stats) { return ia_synthesize_levels(c, a, 1, stats); }

int ia_synthesize_levels(ia_ctx *c, const ia_level_args *args, int n_jobs, ia_stats *stats) {
  if (!c || !args) return fail(IA_EINVAL, "ia_synthesize_level: NULL argument");
  if (n_jobs < 1 || n_jobs > IA_MAX_JOBS)
    return fail(IA_EINVAL, "ia_synthesize_levels: n_jobs must be 1.." + std::to_string(IA_MAX_JOBS));
  const ia_level_args *a = &args[0];
  int rc;
  for (int j = 0; j < n_jobs; j++) {
    const ia_level_args *x = &args[j];
    if ((rc = check_level_args(x))) return rc;
    if (x->ch != a->ch || x->n_ap != a->n_ap || x->a_h != a->a_h || x->a_w != a->a_w || x->b_h != a->b_h ||
        x->b_w != a->b_w || x->mem != a->mem)
      return fail(IA_EINVAL, "ia_synthesize_levels: every job of a batch has the same shapes, channels and mem kind");
    if (x->A != a->A || x->Ac != a->Ac || x->Ap != a->Ap || x->Apc != a->Apc)
      return fail(IA_EINVAL, "ia_synthesize_levels: every job of a batch shares the A side (same A / A' buffers)");
  }
  HIP_TRY(hipSetDevice(c->dev));
  const int J = n_jobs;

  LevelGeo g;
  g.pos2row = nullptr;
  g.ch = a->ch;
  g.D = 55 * a->ch;
  g.KH = kh_for(g.D + 1);
  const int DP = 2 * g.KH;
  g.n_ap = a->n_ap;
  g.ah = a->a_h;
  g.aw = a->a_w;
  g.ahc = (a->a_h + 1) / 2;
  g.awc = (a->a_w + 1) / 2;
  g.bh = a->b_h;
  g.bw = a->b_w;
  g.bhc = (a->b_h + 1) / 2;
  g.bwc = (a->b_w + 1) / 2;
  g.NA = (int64_t)g.n_ap * g.ah * g.aw;
  g.n_tiles = (int)((g.NA + IA_TILE - 1) / IA_TILE);
  // DB shards: over the ranks of ia_comm_init (world > 1), or emulated on this device (option
  // "shard_emulate" = W: the W shards' scans and per-shard certified winners run here one after
  // the other, then the multi-rank finish; no RCCL).  Levels under 64 tiles per shard replicate.
  // Only levels that run the pruned scan are sharded by default: the unpruned scan of a 512^2 or
  // smaller DB gains nothing from 1/W of the tiles once the exchange is paid (DESIGN.md §7,
  // profiles/r03/shard); option "shard_unpruned" = 1 shards those too (tests, very large DBs).
  const bool shard_here = c->shard_unpruned ||
                          (c->prune && c->matcher == IA_MATCH_F16X3 && g.ch == 1 && g.NA >= c->prune_min_rows);
  const bool sharded = shard_here && shard_level(g.n_tiles, c->world);
  const bool emulated = shard_here && !sharded && c->world == 1 && c->shard_emulate > 1 &&
                        shard_level(g.n_tiles, c->shard_emulate);
  const int Wsh = sharded ? c->world : emulated ? c->shard_emulate : 1;  // shards of this level
  const bool multi = Wsh > 1;
  const bool xchg = multi && c->exchange == 1;  // peer-write winner exchange (k_merge_xchg)
  // owner-computes sharded step (exchange = 2, ia_internal.h XOLayout): a rank brings its own
  // job (emulated: one job per shard); checked against the pruned scan below
  const bool xo = multi && c->exchange == 2;
  if (xo) {
    if (sharded && !c->xpeer[0]) return fail(IA_EINVAL, "ia_synthesize_level: exchange = 2 needs ia_xchg_open");
    if (Wsh > IA_XCHG_MAXW) return fail(IA_EINVAL, "ia_synthesize_level: the owner exchange takes <= 16 shards");
    if (sharded && J != 1) return fail(IA_EINVAL, "ia_synthesize_level: exchange = 2 takes the rank's own job (n_jobs = 1)");
    if (emulated && J != Wsh)
      return fail(IA_EINVAL, "ia_synthesize_levels: emulated exchange = 2 takes one job per shard (n_jobs = shard_emulate)");
    if (emulated && (rc = xchg_alloc(c, Wsh))) return rc;
    if ((rc = c->xo_inv.ensure((size_t)IA_XO_MAXT * IA_TILE * 4))) return rc;
    HIP_TRY(hipMemsetAsync(c->xerr.p, 0, 4, c->st));
  }
  if (xchg) {
    if (sharded && !c->xpeer[0]) return fail(IA_EINVAL, "ia_synthesize_level: exchange = 1 needs ia_xchg_open");
    if (Wsh > IA_XCHG_MAXW) return fail(IA_EINVAL, "ia_synthesize_level: the peer-write exchange takes <= 16 shards");
    if (emulated && (rc = xchg_alloc(c, Wsh))) return rc;
    if ((int64_t)std::min(g.bh, (g.bw + 2) / 3) * J > IA_XCHG_MAXQ)
      return fail(IA_EINVAL, "ia_synthesize_level: wavefront steps (all jobs) wider than the exchange slots");
    HIP_TRY(hipMemsetAsync(c->xerr.p, 0, 4, c->st));
  }
  for (int j = 0; j < J; j++)
    if (multi && args[j].dbg_src)
      return fail(IA_EINVAL, "ia_synthesize_level: debug outputs are produced by single-rank levels only");
  {
    int64_t t0 = 0, t1 = g.n_tiles;  // this rank's contiguous DB tiles (unpruned sharded levels hold only those)
    if (sharded) ia_shard_tiles(g.NA, c->world, c->rank, &t0, &t1);
    g.tile0 = (int)t0;
    g.tile1 = (int)t1;
  }

  const size_t nA = (size_t)g.ah * g.aw * g.ch, nAc = (size_t)g.ahc * g.awc * g.ch;
  const size_t nB = (size_t)g.bh * g.bw * g.ch, nBc = (size_t)g.bhc * g.bwc * g.ch;
  const int64_t NB = (int64_t)g.bh * g.bw;
  const void *dA, *dAc, *dAp, *dApc;
  if ((rc = stage(c, c->A, a->A, nA * 8, a->mem, &dA)) || (rc = stage(c, c->Ac, a->Ac, nAc * 8, a->mem, &dAc)) ||
      (rc = stage(c, c->Ap, a->Ap, nA * g.n_ap * 8, a->mem, &dAp)) ||
      (rc = stage(c, c->Apc, a->Apc, nAc * g.n_ap * 8, a->mem, &dApc)))
    return rc;
  // the B side of every job (host buffers: one staging set per job)
  if ((int)c->jb.size() < J) c->jb.resize(J);
  std::vector<JobPtrs> jp(J);
  for (int j = 0; j < J; j++) {
    const ia_level_args *x = &args[j];
    JobBufs &b = c->jb[j];
    const void *dB, *dBc, *dBpc, *dW;
    if ((rc = stage(c, b.B, x->B, nB * 8, x->mem, &dB)) || (rc = stage(c, b.Bc, x->Bc, nBc * 8, x->mem, &dBc)) ||
        (rc = stage(c, b.Bpc, x->Bpc, nBc * 8, x->mem, &dBpc)) || (rc = stage(c, b.W, x->weights, (size_t)g.D * 8, x->mem, &dW)) ||
        (rc = b.pstat.ensure((size_t)NB * 4)))
      return rc;
    JobPtrs &p = jp[j];
    p.Bc = (const double *)dBc;
    p.B = (const double *)dB;
    p.Bpc = (const double *)dBpc;
    p.weights = (const double *)dW;
    p.kf = x->kappa_factor;
    p.pstat = b.pstat.as<unsigned>();
    if (x->mem == IA_MEM_DEVICE) {
      p.Bp = x->Bp;
      p.s = x->s_out;
      p.im = x->im_out;
      p.dbg_src = x->dbg_src;
      p.dbg_dist = x->dbg_dist;
    } else {
      if ((rc = b.Bp.ensure(nB * 8)) || (rc = b.S.ensure((size_t)NB * 8)) || (rc = b.IM.ensure((size_t)NB * 4))) return rc;
      p.Bp = b.Bp.as<double>();
      p.s = b.S.as<int32_t>();
      p.im = b.IM.as<int32_t>();
      HIP_TRY(hipMemcpyAsync(p.Bp, x->Bp, nB * 8, hipMemcpyHostToDevice, c->st));
      p.dbg_src = nullptr;
      p.dbg_dist = nullptr;
      if (x->dbg_src) {
        if ((rc = b.DSRC.ensure((size_t)NB * 24)) || (rc = b.DDIST.ensure((size_t)NB * 16))) return rc;
        p.dbg_src = b.DSRC.as<int32_t>();
        p.dbg_dist = b.DDIST.as<double>();
      }
    }
    HIP_TRY(hipMemsetAsync(p.pstat, 0, (size_t)NB * 4, c->st));
  }

  // matcher: split-f16 when the channel count has a K3h instance and every image value fits
  // (IA_F16_MAXABS, one 4-byte read-back per level); otherwise the fp32 MFMA scan
  bool use_h = false;
  if (c->matcher == IA_MATCH_F16X3 && ia_ks_for(g.ch) > 0) {
    if ((rc = c->absmax.ensure(4))) return rc;
    HIP_TRY(hipMemsetAsync(c->absmax.p, 0, 4, c->st));
    for (int j = 0; j < J; j++) {
      const double *arrs[8] = {j ? nullptr : (const double *)dA, j ? nullptr : (const double *)dAc,
                               j ? nullptr : (const double *)dAp, j ? nullptr : (const double *)dApc,
                               jp[j].B, jp[j].Bc, jp[j].Bpc, jp[j].Bp};
      const int64_t ns8[8] = {(int64_t)nA, (int64_t)nAc, (int64_t)(nA * g.n_ap), (int64_t)(nAc * g.n_ap),
                              (int64_t)nB, (int64_t)nBc, (int64_t)nBc, (int64_t)nB};
      ia_launch_absmax(arrs, ns8, c->absmax.as<unsigned>(), c->st);
    }
    unsigned mbits = 0;
    HIP_TRY(hipMemcpyAsync(&mbits, c->absmax.p, 4, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    float mx;
    std::memcpy(&mx, &mbits, 4);
    use_h = mx <= IA_F16_MAXABS;
  }
  g.KS = use_h ? ia_ks_for(g.ch) : 0;
  // certified pruned scan (1 channel, large DBs; every query of a step sorted in one
  // workgroup's LDS)
  int64_t T, Mmax;
  ia_wavefront_shape(g.bh, g.bw, &T, &Mmax);
  const int64_t Mtmax = Mmax * J;  // queries of the widest step over all jobs
  // (exchange = 2 emulated: each owner's queries at its own tile-aligned offset j Mpad_j)
  const int64_t Mpad_max = std::max((Mtmax + IA_TILE - 1) / IA_TILE * IA_TILE,
                                    xo ? J * ((Mmax + IA_TILE - 1) / IA_TILE * IA_TILE) : 0);
  const bool prune = c->prune && use_h && g.ch == 1 && g.NA >= c->prune_min_rows && Mpad_max <= 4096 &&
                     (g.n_tiles + c->scan_wgs - 1) / c->scan_wgs <= IA_K3P_MAXK_LDS;
  // option "nn_bound": per-pixel exact NN rows of a pruned one-rank level (-1 until merged)
  for (int j = 0; j < J; j++) {
    jp[j].nn = nullptr;
    if (prune && c->nn_bound) {  // (every merge form writes it: fused, owner-computes, exchange finishes)
      JobBufs &b = c->jb[j];
      if ((rc = b.NN.ensure((size_t)NB * 4))) return rc;
      jp[j].nn = b.NN.as<int32_t>();
      HIP_TRY(hipMemsetAsync(jp[j].nn, 0xFF, (size_t)NB * 4, c->st));
    }
  }
  if ((rc = c->jobs.ensure(sizeof(JobPtrs) * J))) return rc;
  HIP_TRY(hipMemcpyAsync(c->jobs.p, jp.data(), sizeof(JobPtrs) * J, hipMemcpyHostToDevice, c->st));
  const JobSet djobs{jp[0], c->jobs.as<JobPtrs>(), J};
  if (xo && !prune)
    return fail(IA_EINVAL, "ia_synthesize_level: exchange = 2 shards pruned levels only (1 channel, split-f16, <= 4096 "
                           "queries per step)");
  // owner-computes geometry: per owner QTj query tiles in bpj blocks of QTx tiles, QTs = bpj QTx
  // tiles per owner in the step layout (pads past QTj never contracted)
  int xo_bpj = 1, xo_QTx = 1, xo_QTs = 1;
  if (xo) {
    const int QTj = (int)((Mmax + IA_TILE - 1) / IA_TILE);
    xo_bpj = (QTj + ia_k3h_qtmax(g.KS) - 1) / ia_k3h_qtmax(g.KS);
    xo_QTx = (QTj + xo_bpj - 1) / xo_bpj;
    xo_QTs = xo_bpj * xo_QTx;
    if (Wsh * xo_QTs > IA_XO_MAXT || Wsh * xo_bpj > IA_NWG_H)
      return fail(IA_EINVAL, "ia_synthesize_level: exchange = 2: wavefront steps too wide for the exchange area");
  }
  // Pruned levels: every rank holds the whole Morton-sorted DB, its tiles stored shard by shard
  // (ia_internal.h ia_shard_morton_tile: shard r = Morton tiles r, r + W, ...), and scans its own
  // contiguous storage range.  Unpruned levels: contiguous tile ranges (ia_shard_tiles).
  if (prune) {
    g.tile0 = 0;
    g.tile1 = g.n_tiles;
  }
  const int ns = g.tile1 - g.tile0;  // DB tiles this process holds
  struct Shard {
    int t0, t1, nwg, tpw;  // storage tiles [t0, t1) of the level's DB, scan decomposition
  };
  auto decomp = [&](int t0, int t1) {
    Shard d{t0, t1, 0, 0};
    const int n = t1 - t0;
    if (prune) d.nwg = std::min(c->scan_wgs, n);  // round-robin chunks: WG w owns tiles w + nwg*k
    else {
      d.tpw = use_h ? std::max(IA_WGH / IA_WAVE, (n + c->scan_wgs - 1) / c->scan_wgs) : std::max(4, (n + IA_WG_TARGET - 1) / IA_WG_TARGET);
      d.nwg = (n + d.tpw - 1) / d.tpw;
    }
    return d;
  };
  std::vector<Shard> shards;  // the shards this process scans
  if (!multi) {
    shards.push_back(decomp(g.tile0, g.tile1));
  } else {
    for (int r = sharded ? c->rank : 0; r < (sharded ? c->rank + 1 : Wsh); r++) {
      if (prune) {
        const int t0 = (int)ia_shard_off(g.n_tiles, Wsh, r), t1 = (int)ia_shard_off(g.n_tiles, Wsh, r + 1);
        shards.push_back(decomp(t0, t1));
      } else {
        int64_t t0, t1;
        ia_shard_tiles(g.NA, Wsh, r, &t0, &t1);
        shards.push_back(decomp((int)t0, (int)t1));
      }
    }
  }
  int nwg_max = 1;
  for (const Shard &x : shards) nwg_max = std::max(nwg_max, x.nwg);
  g.nwg = shards[0].nwg;
  g.tiles_per_wg = shards[0].tpw;
  const size_t rec_stride = (size_t)Mtmax * nwg_max;  // records of one shard's scan
  const size_t db_row_bytes = use_h ? (size_t)16 * g.KS * 4 : (size_t)DP * 4;  // hi+lo f16 / fp32 per column
  const size_t tile_bytes = use_h ? (size_t)ia_k3h_tile_bytes(g.KS) : (size_t)IA_TILE * DP * 4;  // one stored DB tile

  // per-level scratch
  if ((rc = c->db.ensure((size_t)std::max(ns, 1) * IA_TILE * db_row_bytes)) || (rc = c->mu.ensure((16 + 4 * 3 * 128) * 8)) ||
      (rc = c->db64.ensure((size_t)g.NA * ia_db64_stride(g.ch) * 8)) ||
      (rc = c->Rbits.ensure(4)) || (rc = c->q64.ensure((size_t)Mpad_max * g.D * 8 * 2)) ||
      (rc = c->qn2.ensure((size_t)Mpad_max * 8 * 2)) || (rc = c->qf.ensure((size_t)Mpad_max * db_row_bytes)) ||
      (rc = c->rec.ensure(rec_stride * shards.size() * 16)) || (rc = c->recT.ensure(rec_stride * shards.size() * 4)) ||
      (rc = c->win.ensure((size_t)Mtmax * 16)) || (rc = c->allwin.ensure((size_t)Mtmax * 16 * Wsh)) ||
      (rc = c->counters.ensure(5 * 8)) ||
      (rc = c->pairs.ensure(6 * IA_NWG_H * 8)) || (rc = c->ord.ensure(2 * 4096 * 4)) ||
      (rc = c->qinfo.ensure(prune ? (size_t)Mpad_max * 3 * 16 * 2 : 16)))
    return rc;
  if (prune && ((rc = c->qs_order.ensure((size_t)Mpad_max * 4)) || (rc = c->qs_info.ensure((size_t)Mpad_max * 3 * 16)) ||
                (rc = c->qs_frag.ensure((size_t)Mpad_max * db_row_bytes)) ||
                (rc = c->qs_tbox.ensure((size_t)Mpad_max / IA_TILE * 3 * 16))))
    return rc;
  // option "stamps" (pruned levels): per-launch workgroup stamps of every K3p launch (<= IA_NWG_H
  // workgroups each) and every fused merge launch (<= Mpad_max + J + 1 workgroups)
  const bool stamped = c->stamps && prune;
  const int64_t k3_cap = T * (int64_t)shards.size() * (c->k3p_blocks ? 1 : 8);
  const int mg_stride = (int)Mpad_max + J + 64;
  const int64_t mg_cap = T * (xo ? J : 1);  // merge launches per step: one, or one per owned job (exchange 2)
  int64_t k3_n = 0, mg_n = 0;
  if (stamped) {
    // the slots start zeroed (fresh buffers here; the slots a level used are cleared after it)
    const size_t k3b = (size_t)k3_cap * IA_NWG_H * 16, mgb = (size_t)mg_cap * mg_stride * 16;
    const bool fresh_k3 = c->stamp_k3.cap < k3b, fresh_mg = c->stamp_mg.cap < mgb;
    if ((rc = c->stamp_k3.ensure(k3b)) || (rc = c->stamp_mg.ensure(mgb)) ||
        (rc = c->stamp_dur.ensure((size_t)(2 * k3_cap + mg_cap) * 16)))
      return rc;
    if (fresh_k3) HIP_TRY(hipMemsetAsync(c->stamp_k3.p, 0, c->stamp_k3.cap, c->st));
    if (fresh_mg) HIP_TRY(hipMemsetAsync(c->stamp_mg.p, 0, c->stamp_mg.cap, c->st));
  }
  auto k3_stamp = [&]() -> unsigned long long * {
    return stamped && k3_n < k3_cap ? c->stamp_k3.as<unsigned long long>() + (size_t)2 * IA_NWG_H * k3_n++ : nullptr;
  };
  auto mg_stamp = [&]() -> unsigned long long * {
    return stamped && mg_n < mg_cap ? c->stamp_mg.as<unsigned long long>() + (size_t)2 * mg_stride * mg_n++ : nullptr;
  };
  // the slots this level wrote are cleared on EVERY exit (an early error return after
  // some stamped launches left non-zero slots that a later, smaller launch would have read)
  struct StampClear {
    ia_ctx *c;
    const int64_t &k3_n, &mg_n;
    int mg_stride;
    ~StampClear() {
      if (k3_n) (void)hipMemsetAsync(c->stamp_k3.p, 0, (size_t)k3_n * IA_NWG_H * 16, c->st);
      if (mg_n) (void)hipMemsetAsync(c->stamp_mg.p, 0, (size_t)mg_n * mg_stride * 16, c->st);
    }
  } stamp_clear{c, k3_n, mg_n, mg_stride};
  double bytes_all_fixed = 0.;  // algorithmic bytes of every pruned launch besides its DB tiles
  double db_cap_all = 0.;       // the whole tiles of every pruned launch's DB range, each counted once
                                // (a launch of nqb query blocks streams a tile once per block)
  // per-workgroup counters of the pruned scan: [pairs | pairs (timed steps) | tiles | tiles (timed) |
  // extra half-tiles | extra half-tiles (timed)][wg]
  HIP_TRY(hipMemsetAsync(c->pairs.p, 0, 6 * IA_NWG_H * 8, c->st));
  HIP_TRY(hipMemsetAsync(c->Rbits.p, 0, 4, c->st));
  HIP_TRY(hipMemsetAsync(c->counters.p, 0, 5 * 8, c->st));

  Imgs Aim{(const double *)dAc, (const double *)dA, (const double *)dApc, (const double *)dAp,
           g.ah, g.aw, g.ahc, g.awc, (int64_t)nA, (int64_t)nAc};
  Imgs Bim{nullptr, nullptr, nullptr, nullptr, g.bh, g.bw, g.bhc, g.bwc, 0, 0};  // images per job (JobPtrs)

  HIP_TRY(hipEventRecord(c->lv0, c->st));
  ia_launch_means(g.ch, Aim, g.n_ap, c->mu.as<double>(), c->st);
  HIP_TRY(hipEventRecord(c->kb[0], c->st));
  ia_launch_db64_build(g, Aim, c->db64.as<double>(), c->st);  // every row: coherence reads any row
  HIP_TRY(hipEventRecord(c->kb[1], c->st));
  double ufac = 0.;
  if (prune && (rc = prepare_prune(c, g, c->mu.as<double>(), Wsh, &ufac)))
    return rc;  // sets g.pos2row
  HIP_TRY(hipEventRecord(c->kb[2], c->st));
  if (ns > 0) {
    if (use_h) ia_launch_db_build_h(g, Aim, c->db64.as<double>(), c->mu.as<double>(), c->db.p, c->Rbits.as<unsigned>(), c->st);
    else ia_launch_db_build(g, Aim, c->mu.as<double>(), c->db.as<float4>(), c->Rbits.as<unsigned>(), c->st);
  }
  HIP_TRY(hipEventRecord(c->kb[3], c->st));
  HIP_TRY(hipEventRecord(c->lv1, c->st));

  MergeArgs ma;
  ma.db64 = c->db64.as<double>();
  ma.rec = c->rec.as<float4>();
  ma.recT = c->recT.as<float>();
  ma.q64 = c->q64.as<double>();
  ma.qn2 = c->qn2.as<double>();
  ma.Rbits = c->Rbits.as<unsigned>();
  ma.nwg = g.nwg;
  ma.tpw = g.tiles_per_wg;
  ma.pos0 = g.tile0 * IA_TILE;
  ma.pos_end = g.tile1 * IA_TILE;
  ma.NT = g.n_tiles;
  ma.NA = (int)g.NA;
  ma.pos2row = g.pos2row;
  ma.rr = prune ? 1 : 0;
  ma.qinfo = prune ? c->qinfo.as<float4>() : nullptr;
  ma.boxes = prune ? c->boxes.as<float4>() : nullptr;
  ma.ufac = ufac;
  ma.img_rows = (c->row_source == 1 && g.ch == 1) ? 1 : 0;
  ma.eps_c = use_h ? ia_eps_c_h(g.KS, prune || c->k3_variant == 1) : ia_eps_c(DP);
  ma.eps_a = use_h ? ia_eps_a_h() : 0.;
  // per shard: its records, decomposition, DB positions (and table / boxes of a pruned level)
  std::vector<MergeArgs> mas(shards.size(), ma);
  std::vector<int64_t> shard_rows(shards.size(), 0);  // real DB rows in each shard (unpruned flops)
  for (size_t i = 0; i < shards.size(); i++) {
    const Shard &x = shards[i];
    MergeArgs &m = mas[i];
    m.rec = c->rec.as<float4>() + i * rec_stride;
    m.recT = c->recT.as<float>() + i * rec_stride;
    m.nwg = x.nwg;
    m.tpw = x.tpw;
    m.pos0 = x.t0 * IA_TILE;
    m.pos_end = x.t1 * IA_TILE;
    if (prune) {
      m.pos2row = g.pos2row + (size_t)x.t0 * IA_TILE;
      m.boxes = c->boxes.as<float4>() + 2 * (size_t)x.t0;
      m.NT = x.t1 - x.t0;
    }
    for (int t = x.t0; t < x.t1 && !prune; t++) {
      const int64_t tr = ia_tile_perm(t, g.n_tiles);
      shard_rows[i] += std::min<int64_t>(IA_TILE, (g.NA - tr + g.n_tiles - 1) / g.n_tiles);
    }
  }

  const int qtmax = use_h ? ia_k3h_qtmax(g.KS) : ia_k3_qtmax(g.KH);
  const int stride = c->time_dist > 0 ? c->time_dist : 0;
  // fused K4(t) + K2p(t + 1) (option "fuse_gather", ia_kernels.hip k_merge_gather): one-job
  // unsharded pruned levels (<= 256 records per query: one launch's chunks, or nch <= 256 of a
  // wide step's 2-D launch); the query buffers alternate by step parity
  static_assert(IA_NWG_H <= 4 * IA_WAVE, "k_merge_gather reads 4 records per lane");
  // (owner-computes steps too: each local owner's merge + its next gather, which publishes)
  // (batched jobs: one handoff row set per job.  Unpruned levels - K2h fused, option
  // "fuse_unpruned" - measured slower: their longer fused launches delay the pipelined finest
  // level's scans, and cfg5's batched 512^2 steps lose 1-2 %)
  bool chain = c->fuse_gather && use_h && g.ch == 1 && ma.img_rows == 0 && g.bw >= 3 &&
               (prune || c->fuse_unpruned) && ((!multi && !xo && mas[0].nwg <= 4 * IA_WAVE) || (xo && prune));
  // (one-rank levels: the process-wide chained-wave budget, g_chain_waves; a launch holds at most
  // Mpad + J waves: merges, entering rows, pads)
  // Owner-computes levels (exchange 2) take the same reservation: their fused launches chain
  // rows like any other (and wait for peers' records besides, which never depend on a chained
  // wave of this process), so the same budget keeps them deadlock-free
  ChainReservation chain_res;
  if (chain && !chain_res.take((int)(Mpad_max + J) + (xo ? 1 : 0), c->chain_budget)) chain = false;
  if (chain) {
    const int hrows = g.bh * J;  // per job (local owner)
    if (c->hand_rows < hrows) {
      HIP_TRY(hipStreamSynchronize(c->st));
      if (c->hand) hipFree(c->hand);
      c->hand = nullptr;
      c->hand_rows = 0;
      HIP_TRY(hipExtMallocWithFlags((void **)&c->hand, (size_t)hrows * sizeof(HandSlot), hipDeviceMallocUncached));
      HIP_TRY(hipMemset(c->hand, 0, (size_t)hrows * sizeof(HandSlot)));
      HIP_TRY(hipDeviceSynchronize());
      c->hand_rows = hrows;
    }
    if (c->kslot_n < Mpad_max) {  // key slots of the gathers' sort (option "fuse_sort")
      HIP_TRY(hipStreamSynchronize(c->st));
      if (c->kslot) hipFree(c->kslot);
      c->kslot = nullptr;
      c->kslot_n = 0;
      HIP_TRY(hipExtMallocWithFlags((void **)&c->kslot, (size_t)Mpad_max * 8, hipDeviceMallocUncached));
      HIP_TRY(hipMemset(c->kslot, 0, (size_t)Mpad_max * 8));
      HIP_TRY(hipDeviceSynchronize());
      c->kslot_n = (int)Mpad_max;
    }
    if ((rc = c->xerr.ensure(4))) return rc;
    HIP_TRY(hipMemsetAsync(c->xerr.p, 0, 4, c->st));
  }
  // query buffers of step t (chain: parity half t & 1)
  auto qhalf = [&](int64_t t, double *&q64, double *&qn2, float4 *&qinfo) {
    const size_t h = chain && (t & 1) ? 1 : 0;
    q64 = c->q64.as<double>() + h * Mpad_max * g.D;
    qn2 = c->qn2.as<double>() + h * Mpad_max;
    qinfo = prune ? c->qinfo.as<float4>() + h * 3 * Mpad_max : nullptr;
  };
  int64_t gathered = -1;  // the step whose gather the previous fused launch ran
  bool gsort = false;     // ... and that launch also sorted it (option "fuse_sort": no K2s, no in-scan sort)
  // (the gathers' sort waits for every wave of its launch: only while all chained waves in flight
  // fit the resident slots, half the budget)
  const bool fsort = chain && prune && !xo && (c->fuse_sort == 1 || (c->fuse_sort == 2 && Mtmax >= IA_FUSE_SORT_MINQ)) &&
                     g_chain_waves.load() <= c->chain_budget / 2;
  const int64_t n_timed = stride ? (T + stride - 1) / stride : 0;
  for (auto *v : {&c->evs, &c->evg, &c->evm})
    if ((int64_t)v->size() < 2 * n_timed) {
      size_t old = v->size();
      v->resize(2 * n_timed);
      for (size_t i = old; i < v->size(); i++) hipEventCreate(&(*v)[i]);
    }
  // algorithmic bytes of one query's gather (K2h / K2p): its 55*ch features read, (K2p) the 12
  // causal coherence candidates' fp64 rows for U, the fp64 row + MFMA fragments + |q'|^2 (+ K2p's
  // pruning record) written
  const double gq_bytes = 55.0 * g.ch * 8 + (prune ? 12.0 * ia_db64_stride(g.ch) * 8 : 0.) + g.D * 8.0 +
                          (use_h ? 16.0 * g.KS * 4 : DP * 4.0) + 8.0 + (prune ? 48.0 : 0.);
  int64_t n_gm = 0;                        // sampled steps (gather / merge brackets)
  double gather_bytes_timed = 0.;
  int64_t dist_launches = 0, launches_timed = 0, n_rec = 0;
  double dist_flops = 0., flops_timed = 0., pairs_full = 0., tiles_full = 0., bytes_timed_fixed = 0.;
  int ord_n = 0;  // pruned scan (k3p_variant 8): queries in the previous step's key order
  // level pipelining: this level's per-step events (recording) / waits on the previous level
  const int gen = c->p_record ? c->p_gen.load() + 1 : 0;
  std::vector<hipEvent_t> *pev = nullptr;
  if (gen) {
    pev = &c->p_ev[gen % 3];
    while ((int64_t)pev->size() < T) {
      hipEvent_t e;
      HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      pev->push_back(e);
    }
    c->p_enq.store(-1);
    c->p_T.store(T);
    c->p_gen.store(gen);  // published last: a dependent reads p_T / p_enq of this generation after it
  }
  struct PDone {  // every return from here on (errors too) releases the dependents' waits
    ia_ctx *c;
    int g;
    ~PDone() {
      if (g) c->p_done.store(g);
    }
  } pdone{c, gen};
  ia_ctx *dp = c->dep;
  const int dgen = c->dep_gen;
  c->dep = nullptr;  // one level call per ia_pipeline_depend
  c->dep_gen = 0;
  int64_t waited = -1;
  // the previous level's host thread stopped enqueueing (it failed): 120 s without progress of
  // its generation or its enqueued steps (a long but healthy predecessor keeps resetting this)
  auto t_prog = std::chrono::steady_clock::now();
  long long seen_enq = -2;
  int seen_gen = -1;
  auto stalled = [&]() {
    const auto now = std::chrono::steady_clock::now();
    const long long e = dp->p_enq.load();
    const int gn = dp->p_gen.load();
    if (e != seen_enq || gn != seen_gen) {
      seen_enq = e;
      seen_gen = gn;
      t_prog = now;
      return false;
    }
    return now - t_prog > std::chrono::seconds(120);
  };
  auto wait_dep = [&](int64_t t) -> int {
    if (!dp) return IA_OK;
    while (dp->p_gen.load() < dgen && dp->p_done.load() < dgen)  // it has started that level
      if (stalled()) return fail(IA_ECOMM, "pipeline: the previous level did not start");
      else std::this_thread::yield();
    const int64_t need = std::min<int64_t>(t / 2 + 4, dp->p_T.load() - 1);
    if (need <= waited) return IA_OK;
    while (dp->p_done.load() < dgen && dp->p_enq.load() < need)
      if (stalled()) return fail(IA_ECOMM, "pipeline: the previous level stopped enqueueing");
      else std::this_thread::yield();
    if (dp->p_done.load() < dgen) {
      hipEvent_t ev = dp->p_ev[dgen % 3][need];
      // the previous level usually runs far ahead: an event that already completed needs no
      // barrier packet on this stream
      if (hipEventQuery(ev) != hipSuccess) HIP_TRY(hipStreamWaitEvent(c->st, ev, 0));
    }
    waited = need;
    return IA_OK;
  };
  const bool no_events = c->p_last != 0;  // nothing waits on this call's steps
  c->p_last = 0;
  auto mark_step = [&](int64_t t) {
    if (!gen) return;
    if (!no_events) hipEventRecord((*pev)[t], c->st);
    c->p_enq.store(t);
  };
  for (int64_t t = 0; t < T; mark_step(t), t++) {
    if ((rc = wait_dep(t))) return rc;
    StepDesc sd;
    sd.t = (int)t;
    sd.J = J;
    ia_wavefront_step(g.bh, g.bw, t, &sd.r0, &sd.M);
    if (sd.M <= 0) {  // levels narrower than 3 columns have empty steps
      ord_n = 0;
      continue;
    }
    const int Mt = J * sd.M;  // queries of this step over all jobs
    sd.Mpad = (Mt + IA_TILE - 1) / IA_TILE * IA_TILE;
    const bool timed_gm = stride && t % stride == 0;
    if (timed_gm) {
      hipEventRecord(c->evg[2 * n_gm], c->st);
      gather_bytes_timed += gq_bytes * Mt;
    }
    if (xo) {
      // ---- owner-computes sharded step (exchange = 2, ia_internal.h XOLayout): every local owner
      // (a rank: its own job; emulated: job j = owner j, each at its own tile-aligned offset)
      // gathers its queries (K2p) and sorts them into every rank's area (K2s); this process's
      // shard scans (K3p) run for all owners' queries and push their records to the owners; each
      // local owner's fused merge (K4) runs over W nch records per query.  The emulated launches
      // are exactly the ranks' launches, one after the other.
      const unsigned seq = ++c->xseq;
      auto area_s = [&](int p, unsigned sq) -> char * {  // parity base of rank p's area for step seq sq
        return (char *)(sharded ? (void *)c->xpeer[p] : c->xbuf) + ia_xslots_bytes(Wsh) + (size_t)(sq & 1u) * XOLayout::PARITY;
      };
      auto area = [&](int p) -> char * { return area_s(p, seq); };
      char *loc = area(sharded ? c->rank : 0);
      const int Mpj = (sd.M + IA_TILE - 1) / IA_TILE * IA_TILE;  // one owner's padded queries
      // owners whose step fits one launch's query tiles skip K2s: K2p publishes the unsorted
      // queries and each K3p block sorts its owner's queries itself (XOPub)
      const bool ink = Mpj <= ia_k3h_qtmax(g.KS) * IA_TILE && !c->xo_presort;
      const int QTs = ink ? Mpj / IA_TILE : xo_QTs;  // tiles per owner in this step's layout
      const int Mrec = Wsh * QTs * IA_TILE;
      StepDesc s1 = sd;
      s1.J = 1;
      s1.Mpad = Mpj;
      auto owner_of = [&](int jl) { return sharded ? c->rank : jl; };
      double *q64t, *qn2t;
      float4 *qinfot;
      qhalf(t, q64t, qn2t, qinfot);
      for (int jl = 0; jl < J; jl++) {
        const JobSet one{jp[jl], c->jobs.as<JobPtrs>() + jl, 1};
        const size_t q0 = (size_t)jl * Mpj;
        if (chain && gathered == t) {  // K2p (+ publish) ran in the previous step's fused merge
          if (!ink)
            ia_launch_query_sort_xo_owner(c, g, qinfot + 3 * q0, (char *)c->qf.p + q0 * db_row_bytes, sd, owner_of(jl),
                                          QTs, seq, sharded ? Wsh : 1, area);
          continue;
        }
        XOPub xp{};
        if (ink) {
          xp.W = sharded ? Wsh : 1;
          for (int p = 0; p < xp.W; p++) xp.area[p] = area(p);
          xp.slot0 = owner_of(jl) * Mpj;
          xp.seq = seq;
        }
        ia_launch_gather_p(g, s1, Bim, one, c->mu.as<double>(), q64t + q0 * g.D, qn2t + q0,
                           (char *)c->qf.p + q0 * db_row_bytes, c->db64.as<double>(), c->pr_basis.as<double>(), ufac,
                           qinfot + 3 * q0, Aim, ma.img_rows, c->st, &xp);
        if (ink) continue;
        ia_launch_query_sort_xo_owner(c, g, qinfot + 3 * q0, (char *)c->qf.p + q0 * db_row_bytes, sd, owner_of(jl), QTs,
                                      seq, sharded ? Wsh : 1, area);
      }
      if (timed_gm) hipEventRecord(c->evg[2 * n_gm + 1], c->st);
      const int nqb = ink ? Wsh : Wsh * xo_bpj;
      const bool timed = stride && t % stride == 0;
      if (timed) hipEventRecord(c->evs[2 * n_rec], c->st);
      // one chunk count for every shard (the owners' merges index records as shard * nch + chunk
      // and map a chunk back to its tiles with it): from the smallest shard, which every rank
      // computes alike (shards differ by at most one tile, ia_shard_off)
      int nch = std::max(1, std::min((int)(g.n_tiles / Wsh), IA_NWG_H / nqb));
      if (nch >= 64) nch &= ~7;
      for (size_t i = 0; i < shards.size(); i++) {
        const Shard &x = shards[i];
        const int n = x.t1 - x.t0;
        if ((n + nch - 1) / nch > IA_K3P_MAXK_LDS || (int64_t)Wsh * nch * Mrec > IA_XO_MAXREC)
          return fail(IA_EINVAL, "ia_synthesize_level: exchange = 2: shard too large for the pruned scan's chunks");
        XOScan xs{};
        for (int p = 0; p < Wsh; p++) xs.area[p] = sharded ? area(p) : loc;
        xs.flag = reinterpret_cast<const unsigned *>(loc + (ink ? XOLayout::QSEQ : XOLayout::FLAG));
        xs.inv = c->xo_inv.as<int>();
        xs.on = 1;
        xs.s = sharded ? c->rank : (int)i;
        xs.bpj = ink ? 1 : xo_bpj;
        xs.Mrec = Mrec;
        xs.seq = seq;
        xs.err = c->xerr.as<unsigned>();
        xs.timeout_ticks = 2000000000LL;  // 20 s of the 100 MHz s_memrealtime clock
        const char *dbp = (const char *)c->db.p + (size_t)(x.t0 - g.tile0) * tile_bytes;
        const int kv = c->k3p_variant;
        // the in-kernel-sort variant (ink: 20 / 22 / 24) or its presorted form (21 / 25)
        const int k3x = ink ? (kv == 21 ? 20 : kv == 25 ? 24 : kv) : (kv == 25 ? 25 : 21);
        {
            if (ia_launch_k3p(ink ? QTs : xo_QTx, dbp, loc + XOLayout::FRAG, reinterpret_cast<const float4 *>(loc + XOLayout::INFO),
                      mas[i].boxes, mas[i].pos2row, n, 0, sd.M, ink ? Mpj : Mrec, nch, nullptr, nullptr,
                      c->pairs.as<unsigned long long>() + (timed ? IA_NWG_H : 0),
                      c->pairs.as<unsigned long long>() + (timed ? 3 : 2) * IA_NWG_H, k3x, sd.t,
                      reinterpret_cast<const int *>(loc + XOLayout::ORD), 0, sd.r0, nullptr,
                      reinterpret_cast<const float4 *>(loc + XOLayout::TBOX), c->tnorm.as<float>() + x.t0, c->st, nqb,
                      Wsh * QTs, &xs, k3_stamp(), c->rec_wt)) return fail(IA_EINVAL, "pruned scan: no kernel instance for k3p_variant");
          }
        pairs_full += (double)n * Wsh * QTs;
        tiles_full += (double)n * nqb;
        dist_launches++;
        bytes_all_fixed += (double)n * nqb * 32 + (double)Mrec * (16.0 * 16 * g.KS + 48) + (double)Mrec * nch * 24;
        db_cap_all += (double)n * tile_bytes;
        if (timed) {
          launches_timed++;
          bytes_timed_fixed += (double)n * nqb * 32 + (double)Mrec * (16.0 * 16 * g.KS + 48) + (double)Mrec * nch * 24;
        }
      }
      if (timed) hipEventRecord(c->evs[2 * n_rec++ + 1], c->st);
      if (timed_gm) hipEventRecord(c->evm[2 * n_gm], c->st);
      // the next step's layout (fused merge + gather: each owner publishes its next queries)
      const bool fuse_next = chain && t + 1 < T && !(stride && (t % stride == 0 || (t + 1) % stride == 0));
      StepDesc sn{};
      int Mpj_n = 0;
      bool ink_n = false;
      double *q64n = nullptr, *qn2n = nullptr;
      float4 *qinfon = nullptr;
      if (fuse_next) {
        if ((rc = wait_dep(t + 1))) return rc;
        sn.t = (int)(t + 1);
        sn.J = 1;
        ia_wavefront_step(g.bh, g.bw, t + 1, &sn.r0, &sn.M);
        Mpj_n = (sn.M + IA_TILE - 1) / IA_TILE * IA_TILE;
        sn.Mpad = Mpj_n;
        ink_n = Mpj_n <= ia_k3h_qtmax(g.KS) * IA_TILE && !c->xo_presort;
        qhalf(t + 1, q64n, qn2n, qinfon);
      }
      for (int jl = 0; jl < J; jl++) {
        const JobSet one{jp[jl], c->jobs.as<JobPtrs>() + jl, 1};
        const size_t q0 = (size_t)jl * Mpj;
        MergeArgs mx = ma;
        mx.q64 = q64t + q0 * g.D;
        mx.qn2 = qn2t + q0;
        mx.qinfo = qinfot + 3 * q0;
        mx.rec = reinterpret_cast<const float4 *>(loc + XOLayout::REC);
        mx.xo_rts = reinterpret_cast<const unsigned long long *>(loc + XOLayout::RTS);
        mx.nwg = Wsh * nch;
        mx.rr = 1;
        mx.NT = g.n_tiles;
        mx.boxes = c->boxes.as<float4>();
        mx.pos2row = g.pos2row;
        mx.xo_inv = c->xo_inv.as<int>();
        mx.xo_W = Wsh;
        mx.xo_nch = nch;
        mx.xo_Mrec = Mrec;
        mx.xo_o0 = owner_of(jl);
        mx.xo_M = sd.M;
        mx.xo_QTs = QTs;
        mx.xo_seq = seq;
        mx.xo_err = c->xerr.as<unsigned>();
        mx.xo_timeout = 2000000000LL;
        mx.stamp = mg_stamp();
        if (!fuse_next) {
          ia_launch_merge(g, s1, Aim, mx, c->win.as<Winner>(), one, true, c->st);
          continue;
        }
        const size_t q0n = (size_t)jl * Mpj_n;
        NextStep nx{};
        nx.sn = sn;
        nx.q64 = q64n + q0n * g.D;
        nx.qn2 = qn2n + q0n;
        nx.qinfo = qinfon + 3 * q0n;
        nx.qf = (char *)c->qf.p + q0n * db_row_bytes;
        nx.mu = c->mu.as<double>();
        nx.basis = c->pr_basis.as<double>();
        nx.ufac = ufac;
        nx.hand = c->hand + (size_t)jl * g.bh;
        nx.seq = ++c->hseq;
        nx.err = c->xerr.as<unsigned>();
        nx.timeout_ticks = 2000000000LL;
        nx.prefetch = c->prefetch_next;
        nx.early = c->early_gather;
        if (ink_n) {  // the next step's queries go straight to every rank's area (else its K2s sorts them)
          nx.xp.W = sharded ? Wsh : 1;
          for (int p = 0; p < nx.xp.W; p++) nx.xp.area[p] = area_s(p, seq + 1);
          nx.xp.slot0 = owner_of(jl) * Mpj_n;
          nx.xp.seq = seq + 1;
          if (sharded && c->xo_wait && jl == J - 1) {  // ranks: wait here for every owner's next queries
            nx.wait_seq = reinterpret_cast<const unsigned *>(area_s(c->rank, seq + 1) + XOLayout::QSEQ);
            nx.wait_n = Wsh * Mpj_n;
          }
        }
        ia_launch_merge_gather(g, s1, Aim, mx, one, Bim, nx, true, c->st);
      }
      if (fuse_next) gathered = t + 1;
      if (timed_gm) hipEventRecord(c->evm[2 * n_gm++ + 1], c->st);
      continue;
    }
    double *q64t, *qn2t;
    float4 *qinfot;
    qhalf(t, q64t, qn2t, qinfot);
    if (chain) {
      mas[0].q64 = q64t;
      mas[0].qn2 = qn2t;
      mas[0].qinfo = qinfot;
    }
    if (chain && gathered == t)
      ;  // this step's gather ran in the previous step's fused merge
    else if (prune)
      ia_launch_gather_p(g, sd, Bim, djobs, c->mu.as<double>(), q64t, qn2t, c->qf.p, c->db64.as<double>(),
                         c->pr_basis.as<double>(), ufac, qinfot, Aim, ma.img_rows, c->st);
    else if (use_h)
      ia_launch_gather_h(g, sd, Bim, djobs, c->mu.as<double>(), q64t, qn2t, c->qf.p, c->st);
    else
      ia_launch_gather(g, sd, Bim, djobs, c->mu.as<double>(), c->q64.as<double>(), c->qn2.as<double>(), c->qf.as<float>(),
                       c->st);
    if (timed_gm) hipEventRecord(c->evg[2 * n_gm + 1], c->st);
    // pruned scan: queries sorted once per step (K2s) when the step is wider than the in-kernel
    // sort of v6/v7 (512) or variant 11 is selected
    // (variants 11, 12: presorted; 7, 13: in-kernel sort up to 512 queries, presorted v11 / v12 above)
    const int kv = c->k3p_variant;
    // steps wider than one launch's query tiles take the presorted form too when their blocks
    // run as one launch (k3p_blocks): one K2s launch instead of a second scan launch
    const bool wide = sd.Mpad > 512 || (c->k3p_blocks && sd.Mpad > qtmax * IA_TILE);
    // sorted by the previous launch's gathers: the presorted form of the variant, no K2s
    const bool gsorted = fsort && gathered == t && gsort;
    // wide steps: the presorted form of the variant - under 24 that is 25, the two-pass form
    // (round 6, on the trimmed stream: cfg4 6.66 -> 6.91 M px/s against 21's whole tiles; round 4's
    // kernels had it the other way), under 20 / 22 it is 21
    const int k3v = (kv == 21 || kv == 25) ? kv : (prune && (wide || gsorted) ? (kv == 24 ? 25 : 21) : kv);
    const bool presorted = k3v == 21 || k3v == 25;
    const float4 *tboxp = gsorted ? nullptr : c->qs_tbox.as<float4>();  // nullptr: boxes from the slice
    if (prune && presorted && !gsorted)
      ia_launch_query_sort(qinfot, c->qf.p, sd.Mpad, g.KS, c->qs_order.as<int>(), c->qs_info.as<float4>(),
                           c->qs_frag.p, c->qs_tbox.as<float4>(), c->st);
    if (ns > 0) {
      const int qtt = sd.Mpad / IA_TILE, nqb = (qtt + qtmax - 1) / qtmax;
      const bool timed = stride && t % stride == 0;
      if (timed) hipEventRecord(c->evs[2 * n_rec], c->st);
      for (size_t i = 0; i < shards.size(); i++) {
        const Shard &x = shards[i];
        MergeArgs &m = mas[i];
        const int n = x.t1 - x.t0;
        const char *dbp = (const char *)c->db.p + (size_t)(x.t0 - g.tile0) * tile_bytes;
        m.nwg = x.nwg;
        if (prune && presorted && nqb > 1 && c->k3p_blocks) {
          // one launch for all query blocks (option "k3p_blocks"): nqb blocks x nch DB chunks of
          // the shard, nch a multiple of 8 (the blocks of a chunk on one XCD) when that loses
          // little; records per query = nch, the merge's chunk count for this step
          int nch = std::max(1, std::min(n, IA_NWG_H / nqb));
          if (nch >= 64) nch &= ~7;
          if ((n + nch - 1) / nch <= IA_K3P_MAXK_LDS) {
            const int qtb = (qtt + nqb - 1) / nqb;
            const float *tn = c->tnorm.as<float>() + x.t0;
            {
            if (ia_launch_k3p(qtb, dbp, c->qs_frag.p, c->qs_info.as<float4>(), m.boxes, m.pos2row, n, 0, Mt, sd.Mpad, nch,
                          (float4 *)m.rec, (float *)m.recT, c->pairs.as<unsigned long long>() + (timed ? IA_NWG_H : 0),
                          c->pairs.as<unsigned long long>() + (timed ? 3 : 2) * IA_NWG_H, k3v, sd.t, c->qs_order.as<int>(),
                          0, sd.r0, nullptr, tboxp, tn, c->st, nqb, qtt, nullptr, k3_stamp(), c->rec_wt)) return fail(IA_EINVAL, "pruned scan: no kernel instance for k3p_variant");
          }
            m.nwg = nch;
            pairs_full += (double)n * qtt;
            tiles_full += (double)n * nqb;
            dist_launches++;
            bytes_all_fixed += (double)n * nqb * 32 + (double)sd.Mpad * (16.0 * 16 * g.KS + 48) + (double)Mt * nch * 20;
            db_cap_all += (double)n * tile_bytes;
            if (timed) {
              launches_timed++;
              bytes_timed_fixed += (double)n * nqb * 32 + (double)sd.Mpad * (16.0 * 16 * g.KS + 48) + (double)Mt * nch * 20;
            }
            continue;
          }
        }
        int qt0 = 0;
        for (int b = 0; b < nqb; b++) {
          const int qt = qtt / nqb + (b < qtt % nqb ? 1 : 0);
          const float *tn = prune ? c->tnorm.as<float>() + x.t0 : nullptr;
          if (prune && presorted)
            {
            if (ia_launch_k3p(qt, dbp, c->qs_frag.p, c->qs_info.as<float4>(), m.boxes, m.pos2row, n, qt0, Mt, sd.Mpad, x.nwg,
                          (float4 *)m.rec, (float *)m.recT, c->pairs.as<unsigned long long>() + (timed ? IA_NWG_H : 0),
                          c->pairs.as<unsigned long long>() + (timed ? 3 : 2) * IA_NWG_H, k3v, sd.t,
                          c->qs_order.as<int>(), 0, sd.r0, nullptr, tboxp, tn, c->st, 1, 0, nullptr, k3_stamp(), c->rec_wt)) return fail(IA_EINVAL, "pruned scan: no kernel instance for k3p_variant");
          }
          else if (prune)
            {
            if (ia_launch_k3p(qt, dbp, c->qf.p, qinfot, m.boxes, m.pos2row, n, qt0, Mt, sd.Mpad, x.nwg,
                          (float4 *)m.rec, (float *)m.recT, c->pairs.as<unsigned long long>() + (timed ? IA_NWG_H : 0),
                          c->pairs.as<unsigned long long>() + (timed ? 3 : 2) * IA_NWG_H,
                          k3v, sd.t, c->ord.as<int>() + (sd.t & 1 ? 0 : 4096), ord_n, sd.r0,
                          c->ord.as<int>() + (sd.t & 1 ? 4096 : 0), nullptr, tn, c->st, 1, 0, nullptr, k3_stamp(), c->rec_wt)) return fail(IA_EINVAL, "pruned scan: no kernel instance for k3p_variant");
          }
          else if (use_h)
            ia_launch_k3h(g.KS, qt, dbp, c->qf.p, n, x.tpw, qt0, Mt, x.nwg, m.pos0, g.n_tiles, (float4 *)m.rec,
                          (float *)m.recT, c->k3_variant, c->st);
          else
            ia_launch_k3(g.KH, qt, (const float4 *)dbp, c->qf.as<float4>(), n, x.tpw, qt0, Mt, x.nwg, m.pos0, g.n_tiles,
                         (float4 *)m.rec, (float *)m.recT, c->st);
          const int mq = std::min(Mt, (qt0 + qt) * IA_TILE) - qt0 * IA_TILE;
          const double fl = prune ? 0. : 2.0 * g.D * (double)shard_rows[i] * std::max(mq, 0);  // pruned: pair counters
          dist_flops += fl;
          pairs_full += (double)n * qt;
          tiles_full += (double)n;
          dist_launches++;
          if (prune) {
            bytes_all_fixed += (double)n * 32 + (double)sd.Mpad * (16.0 * 16 * g.KS + 48) + (double)mq * x.nwg * 20;
            db_cap_all += (double)n * tile_bytes;
          }
          if (timed) {
            flops_timed += fl;
            launches_timed++;
            // algorithmic bytes of a pruned launch besides its DB tiles: tile boxes, query
            // fragments and pruning records, K3 records written
            bytes_timed_fixed += (double)n * 32 + (double)sd.Mpad * (16.0 * 16 * g.KS + 48) + (double)mq * x.nwg * 20;
          }
          qt0 += qt;
        }
      }
      if (timed) hipEventRecord(c->evs[2 * n_rec++ + 1], c->st);
      ord_n = prune && J == 1 && !multi && sd.Mpad <= 4096 ? sd.M : 0;
    }
    if (timed_gm) hipEventRecord(c->evm[2 * n_gm], c->st);
    if (!multi && chain && t + 1 < T && !(stride && (t % stride == 0 || (t + 1) % stride == 0))) {
      // this step's merge + the next step's gather (not on sampled steps: their K2 / K4 brackets)
      if ((rc = wait_dep(t + 1))) return rc;  // the next step's gather reads the previous level
      NextStep nx{};
      nx.sn.t = (int)(t + 1);
      nx.sn.J = J;
      ia_wavefront_step(g.bh, g.bw, t + 1, &nx.sn.r0, &nx.sn.M);
      nx.sn.Mpad = (J * nx.sn.M + IA_TILE - 1) / IA_TILE * IA_TILE;
      qhalf(t + 1, nx.q64, nx.qn2, nx.qinfo);
      nx.mu = c->mu.as<double>();
      nx.basis = c->pr_basis.as<double>();
      nx.qf = c->qf.p;
      nx.ufac = ufac;
      nx.hand = c->hand;
      nx.seq = ++c->hseq;
      nx.err = c->xerr.as<unsigned>();
      nx.timeout_ticks = 2000000000LL;  // 20 s of the 100 MHz s_memrealtime clock
      nx.prefetch = c->prefetch_next;
      nx.early = c->early_gather;
      // the gathers also sort step t + 1 into k_query_sort's outputs when every wave of the launch
      // can be resident at once (each gather waits for all of the step's keys): k_merge_gather
      // holds one wave per SIMD (264 VGPRs), 1,024 on the chip; 768 leaves room for the kernels of
      // concurrent (pipelined) levels, which never wait on this one
      const int nw = J * sd.M + J + (nx.sn.Mpad - J * nx.sn.M);
      const bool srt = fsort && nw <= IA_FUSE_SORT_MAXW;
      if (srt) {
        nx.kslot = c->kslot;
        nx.sorder = c->qs_order.as<int>();
        nx.sinfo = c->qs_info.as<float4>();
        nx.sfrag = c->qs_frag.p;
      }
      mas[0].stamp = mg_stamp();
      ia_launch_merge_gather(g, sd, Aim, mas[0], djobs, Bim, nx, prune, c->st);
      gathered = t + 1;
      gsort = srt;
    } else if (!multi) {
      mas[0].stamp = mg_stamp();
      ia_launch_merge(g, sd, Aim, mas[0], c->win.as<Winner>(), djobs, true, c->st);
    } else if (xchg) {
      // one-shot peer-write exchange fused into the merge: each shard's winner goes into every
      // rank's buffer; the last launch of this process waits for all W and finishes the pixels
      XchgArgs xa;
      for (int p = 0; p < IA_XCHG_MAXW; p++) xa.peer[p] = sharded ? c->xpeer[p] : (XSlot *)c->xbuf;
      xa.local = sharded ? c->xpeer[c->rank] : (XSlot *)c->xbuf;
      xa.W = Wsh;
      xa.seq = ++c->xseq;
      xa.err = c->xerr.as<unsigned>();
      xa.timeout_ticks = 2000000000LL;  // 20 s of the 100 MHz s_memrealtime clock
      for (size_t i = 0; i < shards.size(); i++) {
        xa.rank = sharded ? c->rank : (int)i;
        ia_launch_merge_xchg(g, sd, Aim, mas[i], xa, djobs, i + 1 == shards.size(), c->st);
      }
    } else {
      // certified per-shard winners, then the global winner (smallest exact distance, lowest row)
      // and coherence / kappa / writeback, identical on every rank
      for (size_t i = 0; i < shards.size(); i++)
        ia_launch_merge(g, sd, Aim, mas[i], (sharded ? c->win.as<Winner>() : c->allwin.as<Winner>() + i * Mt), djobs,
                        false, c->st);
      if (sharded)
        NCCL_TRY(ncclAllGather(c->win.p, c->allwin.p, (size_t)Mt * sizeof(Winner), ncclUint8, c->comm, c->st));
      ia_launch_finish(g, sd, Aim, c->db64.as<double>(), c->q64.as<double>(), c->allwin.as<Winner>(), Wsh, Mt, djobs,
                       c->st);
    }
    if (timed_gm) hipEventRecord(c->evm[2 * n_gm++ + 1], c->st);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(c->lv2, c->st));
  if (stamped) {  // per-launch device ticks: K3p launches first, then the merges
    ia_launch_stamp_durations(c->stamp_k3.as<unsigned long long>(), (int)k3_n, IA_NWG_H, c->stamp_dur.as<unsigned long long>(),
                              c->st, c->stamp_dur.as<unsigned long long>() + 2 * (k3_n + mg_n));
    ia_launch_stamp_durations(c->stamp_mg.as<unsigned long long>(), (int)mg_n, mg_stride,
                              c->stamp_dur.as<unsigned long long>() + 2 * k3_n, c->st);
    // (the slots this level wrote are cleared by stamp_clear when the call returns)
  }
  if (stats)
    for (int j = 0; j < J; j++) ia_launch_reduce_stats(jp[j].pstat, NB, c->counters.as<unsigned long long>(), c->st);
  for (int j = 0; j < J; j++) {
    const ia_level_args *x = &args[j];
    if (x->mem != IA_MEM_HOST) continue;
    HIP_TRY(hipMemcpyAsync(x->Bp, jp[j].Bp, nB * 8, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipMemcpyAsync(x->s_out, jp[j].s, (size_t)NB * 8, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipMemcpyAsync(x->im_out, jp[j].im, (size_t)NB * 4, hipMemcpyDeviceToHost, c->st));
    if (x->dbg_src) {
      HIP_TRY(hipMemcpyAsync(x->dbg_src, jp[j].dbg_src, (size_t)NB * 24, hipMemcpyDeviceToHost, c->st));
      HIP_TRY(hipMemcpyAsync(x->dbg_dist, jp[j].dbg_dist, (size_t)NB * 16, hipMemcpyDeviceToHost, c->st));
    }
  }
  HIP_TRY(hipStreamSynchronize(c->st));
#if IA_PROBE & 16
  if (prune) ia_k3p_probe_dump();
#endif
  if (chain) {
    unsigned xe = 0;
    HIP_TRY(hipMemcpy(&xe, c->xerr.p, 4, hipMemcpyDeviceToHost));
    if (xe & 16) return fail(IA_EHIP, "ia_synthesize_level: a fused gather's handoff did not arrive within 20 s");
  }
  if (xchg || xo) {
    unsigned xe = 0;
    HIP_TRY(hipMemcpy(&xe, c->xerr.p, 4, hipMemcpyDeviceToHost));
    if (xe)
      return fail(IA_ECOMM, std::string("ia_synthesize_level: a peer's ") +
                                (xe & 4 ? "sorted queries" : xe & 8 ? "scan records" : "shard winner") +
                                " did not arrive within 20 s (peer-write exchange)");
  }
  if (stats) {
    unsigned long long ctr[5], prs[4], pfull = 0, ptp = 0, ext[2] = {0, 0};
    HIP_TRY(hipMemcpy(ctr, c->counters.p, sizeof(ctr), hipMemcpyDeviceToHost));
    {  // per-workgroup counter slots (no same-address atomics in the distance kernel)
      std::vector<unsigned long long> slots(6 * IA_NWG_H);
      HIP_TRY(hipMemcpy(slots.data(), c->pairs.p, slots.size() * 8, hipMemcpyDeviceToHost));
      for (int j = 0; j < 4; j++) {
        prs[j] = 0;
        for (int w = 0; w < IA_NWG_H; w++) {
          const unsigned long long v = slots[j * IA_NWG_H + w];
          if (j < 2) {  // pair slots: (pairs with corrections << 32) + pairs (k3p_variant 14/15)
            prs[j] += v & 0xffffffffull;
            pfull += v >> 32;
          } else {  // tile slots: (tiles with a filter-passing block << 32) + tiles loaded
            prs[j] += v & 0xffffffffull;
            ptp += v >> 32;
          }
        }
      }
      for (int w = 0; w < IA_NWG_H; w++) {  // DB half-tiles loaded besides one per loaded tile
        ext[0] += slots[4 * IA_NWG_H + w];
        ext[1] += slots[5 * IA_NWG_H + w];
      }
    }
    const double pair_flops = 2.0 * g.D * IA_TILE * IA_TILE;  // one (DB tile, query tile) pair
    // algorithmic DB bytes of the pruned scan, as each launch's kernel counted them (ADVICE r4:
    // steps wider than 512 queries run another variant than the option names): one half tile
    // (hi or lo) per loaded tile + the extra halves (whole tiles: the lo halves; hi-only stream:
    // the lo halves of the filter-passing tiles; two passes: the passing tiles again, whole)
    auto tile_stream_bytes = [&](double tiles, double extra) { return 0.5 * ia_k3h_tile_bytes(g.KS) * (tiles + extra); };
    if (prune) {
      dist_flops = pair_flops * (double)(prs[0] + prs[1]);
      flops_timed = pair_flops * (double)prs[1];
    }
    stats->pruned_levels += prune ? J : 0;
    stats->dist_pairs += prune ? (double)(prs[0] + prs[1]) : pairs_full;
    stats->dist_pairs_full += pairs_full;
    stats->dist_tiles += prune ? (double)(prs[2] + prs[3]) : tiles_full;
    stats->dist_tiles_full += tiles_full;
    stats->dist_pairs_corrected += (double)pfull;
    stats->dist_tiles_rows += (double)ptp;
    float ms_db = 0.f, ms_syn = 0.f, ms_k1b = 0.f, ms_k1 = 0.f;
    hipEventElapsedTime(&ms_db, c->lv0, c->lv1);
    hipEventElapsedTime(&ms_syn, c->lv1, c->lv2);
    hipEventElapsedTime(&ms_k1b, c->kb[0], c->kb[1]);
    hipEventElapsedTime(&ms_k1, c->kb[2], c->kb[3]);
    if (g.NA >= stats->build_rows) {  // K1b: A-side images read once, every fp64 row written; K1: this
                                      // process's rows read, tiles written (the largest level seen)
      if (g.NA > stats->build_rows) {
        stats->k1b_ms = stats->k1b_bytes = stats->k1_ms = stats->k1_bytes = 0.;
        stats->build_levels = 0;
        stats->build_rows = g.NA;
      }
      const int DSb = ia_db64_stride(g.ch);
      stats->k1b_ms += ms_k1b;
      stats->k1b_bytes += (double)(nA + nAc) * (1 + g.n_ap) * 8 + (double)g.NA * DSb * 8;
      if (ns > 0 && use_h) {
        stats->k1_ms += ms_k1;
        stats->k1_bytes += (double)std::min<int64_t>((int64_t)ns * IA_TILE, g.NA) * DSb * 8 + (double)ns * tile_bytes;
      }
      stats->build_levels += 1;
    }
    for (int64_t i = 0; i < n_gm; i++) {
      float mg = 0.f, mm = 0.f;
      hipEventElapsedTime(&mg, c->evg[2 * i], c->evg[2 * i + 1]);
      hipEventElapsedTime(&mm, c->evm[2 * i], c->evm[2 * i + 1]);
      stats->gather_ms_timed += mg;
      stats->merge_ms_timed += mm;
    }
    stats->gather_launches_timed += n_gm;
    stats->merge_launches_timed += n_gm;
    stats->gather_bytes_timed += gather_bytes_timed;
    stats->pixels += NB * J;
    stats->steps += T;
    stats->reranked += (int64_t)ctr[0];
    stats->fallbacks += (int64_t)ctr[1];
    stats->coherence_wins += (int64_t)ctr[2];
    stats->bound_violations += (int64_t)ctr[3];
    stats->kappa_ambiguous += (int64_t)ctr[4];
    stats->f16_levels += use_h ? J : 0;
    stats->db_ms += ms_db;
    stats->synth_ms += ms_syn;
    stats->dist_launches += dist_launches;
    stats->dist_flops += dist_flops;
    // the pruned scan's timing fields (prune_*, k3p_*, merge_stamp_*, stamp_*) describe the
    // pruned levels with the largest DB seen (prune_rows: the bench's finest level), like k1*_ms
    bool prune_acc = false;
    if (prune && g.NA >= stats->prune_rows) {
      if (g.NA > stats->prune_rows) {
        stats->prune_ms_timed = stats->prune_flops_timed = stats->prune_bytes_timed = 0.;
        stats->prune_launches_timed = 0;
        stats->k3p_stamp_ms = stats->k3p_bytes_all = stats->merge_stamp_ms = stats->stamp_gap_ms = stats->stamp_window_ms = 0.;
        stats->k3p_stamp_start_ms = stats->k3p_stamp_wg_ms = stats->stamp_gap_sm_ms = 0.;
        stats->stamp_gaps_sm = 0;
        stats->k3p_stamp_launches = stats->merge_stamp_launches = stats->stamp_gaps = 0;
        stats->k3p_bytes_unique_all = 0.;
        stats->prune_rows = g.NA;
      }
      prune_acc = true;
    }
    if (stamped && prune_acc && k3_n + mg_n > 0) {
      if (const char *dp = std::getenv("IA_STAMP_DUMP")) {
        // diagnostic: the raw per-workgroup stamps of this level's launches (K3p: IA_NWG_H slots
        // per launch, merges: mg_stride slots; (start | 1, end) ticks of 100 MHz) appended to a file
        std::vector<unsigned long long> r3((size_t)k3_n * IA_NWG_H * 2), rm((size_t)mg_n * mg_stride * 2);
        HIP_TRY(hipMemcpy(r3.data(), c->stamp_k3.p, r3.size() * 8, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(rm.data(), c->stamp_mg.p, rm.size() * 8, hipMemcpyDeviceToHost));
        if (FILE *f = std::fopen(dp, "ab")) {
          const int64_t hdr[4] = {k3_n, IA_NWG_H, mg_n, mg_stride};
          std::fwrite(hdr, 8, 4, f);
          std::fwrite(r3.data(), 8, r3.size(), f);
          std::fwrite(rm.data(), 8, rm.size(), f);
          std::fclose(f);
        }
      }
      std::vector<unsigned long long> sp((size_t)2 * (k3_n + mg_n));  // (start, end) per launch: K3p, then merges
      HIP_TRY(hipMemcpy(sp.data(), c->stamp_dur.p, sp.size() * 8, hipMemcpyDeviceToHost));
      double tk = 0., tm = 0.;
      for (int64_t i = 0; i < k3_n; i++) tk += (double)(sp[2 * i + 1] - sp[2 * i]);
      for (int64_t i = k3_n; i < k3_n + mg_n; i++) tm += (double)(sp[2 * i + 1] - sp[2 * i]);
      stats->k3p_stamp_ms += tk * 1e-5;  // 100 MHz ticks
      {  // the launches' start spread and mean workgroup duration (k_stamp_durations span2)
        std::vector<unsigned long long> s2((size_t)2 * k3_n);
        HIP_TRY(hipMemcpy(s2.data(), c->stamp_dur.as<unsigned long long>() + 2 * (k3_n + mg_n), s2.size() * 8,
                          hipMemcpyDeviceToHost));
        double ss = 0., sw = 0.;
        for (int64_t i = 0; i < k3_n; i++) {
          ss += (double)s2[2 * i];
          sw += (double)s2[2 * i + 1];
        }
        stats->k3p_stamp_start_ms += ss * 1e-5;
        stats->k3p_stamp_wg_ms += sw * 1e-5;
      }
      stats->k3p_stamp_launches += k3_n;
      stats->merge_stamp_ms += tm * 1e-5;
      stats->merge_stamp_launches += mg_n;
      // one scan and one merge per step (a one-job unsharded level): the idle time of the level's
      // chain between its kernels, scan(t) -> merge(t) and merge(t) -> scan(t + 1)
      if (k3_n == mg_n + 1 || k3_n == mg_n) {
        const unsigned long long *m = sp.data() + 2 * k3_n;
        double gap = 0., gsm = 0.;
        int64_t ng = 0, nsm = 0;
        for (int64_t i = 0; i < mg_n; i++) {
          if (m[2 * i] && sp[2 * i + 1] && m[2 * i] >= sp[2 * i + 1]) {
            gsm += (double)(m[2 * i] - sp[2 * i + 1]);
            nsm++;
          }
          if (i + 1 < k3_n && sp[2 * (i + 1)] && m[2 * i + 1] && sp[2 * (i + 1)] >= m[2 * i + 1]) {
            gap += (double)(sp[2 * (i + 1)] - m[2 * i + 1]);
            ng++;
          }
        }
        stats->stamp_gap_ms += (gap + gsm) * 1e-5;
        stats->stamp_gaps += ng + nsm;
        stats->stamp_gap_sm_ms += gsm * 1e-5;
        stats->stamp_gaps_sm += nsm;
        stats->stamp_window_ms += (double)(std::max(sp[2 * k3_n - 1], m[2 * mg_n - 1]) - sp[0]) * 1e-5;
      }
      const double db_stream = tile_stream_bytes((double)(prs[2] + prs[3]), (double)(ext[0] + ext[1]));
      stats->k3p_bytes_all += db_stream + bytes_all_fixed;
      // unique DB bytes: a launch reads each tile of its range at most once as
      // far as the roofline is concerned, however many query blocks stream it
      stats->k3p_bytes_unique_all += std::min(db_stream, db_cap_all) + bytes_all_fixed;
    }
    if (stride && ns > 0) {
      double tot = 0.;
      for (int64_t i = 0; i < n_rec; i++) {
        float ms = 0.f;
        hipEventElapsedTime(&ms, c->evs[2 * i], c->evs[2 * i + 1]);
        tot += ms;
      }
      stats->dist_ms += tot;
      stats->dist_launches_timed += launches_timed;
      stats->dist_flops_timed += flops_timed;
      if (prune_acc) {  // the pruned scan alone (bench roofline): time, MFMA flops, algorithmic bytes
        stats->prune_ms_timed += tot;
        stats->prune_launches_timed += launches_timed;
        stats->prune_flops_timed += flops_timed;
        stats->prune_bytes_timed += tile_stream_bytes((double)prs[3], (double)ext[1]) + bytes_timed_fixed;
      }
    }
  }
  return IA_OK;
}

// ------------------------------------------------------------------------------------------
// GPU preprocessing: Gaussian pyramid reductions and 3x3 colour matrices
// ------------------------------------------------------------------------------------------
int ia_gaussian_pyramid(ia_ctx *c, const double *img, int h, int w, int ch, int n_reduce, const double *weights7,
                        double *out, int mem) {
  if (!c || !img || !weights7 || (n_reduce > 0 && !out) || h < 1 || w < 1 || ch < 1 || ch > 4 || n_reduce < 0)
    return fail(IA_EINVAL, "ia_gaussian_pyramid: bad arguments");
  if (mem != IA_MEM_HOST && mem != IA_MEM_DEVICE) return fail(IA_EINVAL, "ia_gaussian_pyramid: bad mem kind");
  if (n_reduce == 0) return IA_OK;
  HIP_TRY(hipSetDevice(c->dev));
  const size_t n0 = (size_t)h * w * ch;
  size_t tot = 0;  // doubles of all reduced levels
  {
    int hh = h, ww = w;
    for (int k = 0; k < n_reduce; k++) {
      hh = (hh + 1) / 2;
      ww = (ww + 1) / 2;
      tot += (size_t)hh * ww * ch;
    }
  }
  int rc;
  if ((rc = c->py_in.ensure(n0 * 8)) || (rc = c->py_tmp.ensure(n0 * 8)) || (rc = c->py_sm.ensure(n0 * 8)) ||
      (rc = c->py_mm.ensure(2 * 256 * 8)) || (rc = c->py_out.ensure(std::max<size_t>(tot, 1) * 8)))
    return rc;
  const double *din = img;
  if (mem == IA_MEM_HOST) {
    HIP_TRY(hipMemcpyAsync(c->py_in.p, img, n0 * 8, hipMemcpyHostToDevice, c->st));
    din = c->py_in.as<double>();
  }
  double *dout = mem == IA_MEM_DEVICE ? out : c->py_out.as<double>();
  int hh = h, ww = w;
  const double *src = din;
  double *dst = dout;
  for (int k = 0; k < n_reduce; k++) {
    ia_launch_pyramid_reduce(src, dst, c->py_tmp.as<double>(), c->py_sm.as<double>(), c->py_mm.as<double>(), hh, ww, ch,
                             weights7, c->st);
    src = dst;
    hh = (hh + 1) / 2;
    ww = (ww + 1) / 2;
    dst += (size_t)hh * ww * ch;
  }
  HIP_TRY(hipGetLastError());
  if (mem == IA_MEM_HOST) HIP_TRY(hipMemcpyAsync(out, dout, tot * 8, hipMemcpyDeviceToHost, c->st));
  HIP_TRY(hipStreamSynchronize(c->st));
  return IA_OK;
}

int ia_color_matrix(ia_ctx *c, const double *in, int64_t npx, const double *M9, double *out, int mem) {
  if (!c || !in || !M9 || !out || npx < 0) return fail(IA_EINVAL, "ia_color_matrix: bad arguments");
  if (mem != IA_MEM_HOST && mem != IA_MEM_DEVICE) return fail(IA_EINVAL, "ia_color_matrix: bad mem kind");
  if (npx == 0) return IA_OK;
  HIP_TRY(hipSetDevice(c->dev));
  int rc;
  if ((rc = c->py_mm.ensure(2 * 256 * 8))) return rc;
  HIP_TRY(hipMemcpyAsync(c->py_mm.p, M9, 9 * 8, hipMemcpyHostToDevice, c->st));
  const double *din = in;
  double *dout = out;
  if (mem == IA_MEM_HOST) {
    if ((rc = c->py_in.ensure((size_t)npx * 24)) || (rc = c->py_out.ensure((size_t)npx * 24))) return rc;
    HIP_TRY(hipMemcpyAsync(c->py_in.p, in, (size_t)npx * 24, hipMemcpyHostToDevice, c->st));
    din = c->py_in.as<double>();
    dout = c->py_out.as<double>();
  }
  ia_launch_color3(din, dout, npx, c->py_mm.as<double>(), c->st);
  HIP_TRY(hipGetLastError());
  if (mem == IA_MEM_HOST) HIP_TRY(hipMemcpyAsync(out, dout, (size_t)npx * 24, hipMemcpyDeviceToHost, c->st));
  HIP_TRY(hipStreamSynchronize(c->st));
  return IA_OK;
}

// ------------------------------------------------------------------------------------------
// K3h microbenchmark (kernel tuning): the split-f16 distance scan alone on random operands
// ------------------------------------------------------------------------------------------
int ia_k3_microbench(ia_ctx *c, int64_t n_rows, int M, int reps, double *us_per_launch) {
  if (!c || n_rows < 1 || M < 1 || reps < 1 || !us_per_launch) return fail(IA_EINVAL, "ia_k3_microbench: bad arguments");
  const int KS = ia_ks_for(1), qtmax = ia_k3h_qtmax(KS);
  const int qt = (M + IA_TILE - 1) / IA_TILE;
  if (qt > qtmax) return fail(IA_EINVAL, "ia_k3_microbench: M exceeds one launch");
  if (n_rows >= (int64_t)INT32_MAX) return fail(IA_EINVAL, "ia_k3_microbench: n_rows exceeds int32 row ids");
  HIP_TRY(hipSetDevice(c->dev));
  const int n_tiles = (int)((n_rows + IA_TILE - 1) / IA_TILE);
  const int tpw = std::max(IA_WGH / IA_WAVE, (n_tiles + IA_NWG_H - 1) / IA_NWG_H);
  const int nwg = (n_tiles + tpw - 1) / tpw;
  const size_t row_bytes = (size_t)16 * KS * 4;
  int rc;
  if ((rc = c->db.ensure((size_t)n_tiles * IA_TILE * row_bytes)) || (rc = c->qf.ensure((size_t)qt * IA_TILE * row_bytes)) ||
      (rc = c->rec.ensure((size_t)M * nwg * 16)) || (rc = c->recT.ensure((size_t)M * nwg * 4)))
    return rc;
  ia_launch_fill_random_f16(c->db.p, (int64_t)n_tiles * IA_TILE * row_bytes / 2, 12345u, c->st);
  ia_launch_fill_random_f16(c->qf.p, (int64_t)qt * IA_TILE * row_bytes / 2, 777u, c->st);
  auto launch = [&]() {
    ia_launch_k3h(KS, qt, c->db.p, c->qf.p, n_tiles, tpw, 0, M, nwg, 0, n_tiles, c->rec.as<float4>(), c->recT.as<float>(),
                  c->k3_variant, c->st);
  };
  for (int i = 0; i < 3; i++) launch();
  HIP_TRY(hipEventRecord(c->lv0, c->st));
  for (int i = 0; i < reps; i++) launch();
  HIP_TRY(hipEventRecord(c->lv1, c->st));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->st));
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, c->lv0, c->lv1));
  *us_per_launch = 1e3 * ms / reps;
  return IA_OK;
}

// ------------------------------------------------------------------------------------------
// FLANN-compatible exact index (algorithms.py:56,69,74)
// ------------------------------------------------------------------------------------------
int ia_index_build(ia_ctx *c, const double *pts, int64_t n, int d, ia_index **out) {
  if (!c || !pts || !out || n < 1 || d < 1) return fail(IA_EINVAL, "ia_index_build: bad arguments");
  const int KH = kh_for(d + 1);
  if (KH < 0) return fail(IA_EINVAL, "ia_index_build: d must be <= 167");
  if (n >= (int64_t)INT32_MAX) return fail(IA_EINVAL, "ia_index_build: n exceeds int32 row ids");
  HIP_TRY(hipSetDevice(c->dev));
  ia_index *x = new ia_index();
  x->ctx = c;
  x->n = n;
  x->d = d;
  x->KH = KH;
  x->n_tiles = (int)((n + IA_TILE - 1) / IA_TILE);
  x->tpw = std::max(4, (x->n_tiles + IA_WG_TARGET - 1) / IA_WG_TARGET);
  x->nwg = (x->n_tiles + x->tpw - 1) / x->tpw;
  // column means (host, fixed order): centre the fp32 copy, shrinking the MFMA error bound
  std::vector<double> mu(d, 0.);
  for (int64_t i = 0; i < n; i++)
    for (int f = 0; f < d; f++) mu[f] += pts[i * d + f];
  for (int f = 0; f < d; f++) mu[f] /= (double)n;
  int rc;
  if ((rc = x->pts.ensure((size_t)n * d * 8)) || (rc = x->db.ensure((size_t)x->n_tiles * IA_TILE * 2 * KH * 4)) ||
      (rc = x->mu.ensure((size_t)d * 8)) || (rc = x->Rbits.ensure(4)) || (rc = x->counters.ensure(32))) {
    delete x;
    return rc;
  }
  hipMemcpyAsync(x->pts.p, pts, (size_t)n * d * 8, hipMemcpyHostToDevice, c->st);
  hipMemcpyAsync(x->mu.p, mu.data(), (size_t)d * 8, hipMemcpyHostToDevice, c->st);
  hipMemsetAsync(x->Rbits.p, 0, 4, c->st);
  ia_launch_dense_db(KH, x->pts.as<double>(), n, d, x->n_tiles, x->mu.as<double>(), x->db.as<float4>(),
                     x->Rbits.as<unsigned>(), c->st);
  hipError_t e = hipStreamSynchronize(c->st);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) {
    ia_index_destroy(x);
    return fail(IA_EHIP, std::string("ia_index_build: ") + hipGetErrorString(e));
  }
  *out = x;
  return IA_OK;
}

int ia_index_query(ia_index *x, const double *q, int64_t nq, int64_t *idx_out, double *dist_out) {
  if (!x || !q || !idx_out || nq < 0) return fail(IA_EINVAL, "ia_index_query: bad arguments");
  if (nq == 0) return IA_OK;
  ia_ctx *c = x->ctx;
  HIP_TRY(hipSetDevice(c->dev));
  const int64_t BATCH = 4096;
  const int64_t bmax = std::min(nq, BATCH), bpad = (bmax + IA_TILE - 1) / IA_TILE * IA_TILE;
  const int DP = 2 * x->KH;
  int rc;
  if ((rc = x->q.ensure((size_t)bmax * x->d * 8)) || (rc = x->qn2.ensure((size_t)bpad * 8)) ||
      (rc = x->qf.ensure((size_t)bpad * DP * 4)) || (rc = x->rec.ensure((size_t)bmax * x->nwg * 16)) ||
      (rc = x->recT.ensure((size_t)bmax * x->nwg * 4)) || (rc = x->idx.ensure((size_t)bmax * 8)) ||
      (rc = x->dist.ensure((size_t)bmax * 8)))
    return rc;
  HIP_TRY(hipMemsetAsync(x->counters.p, 0, 32, c->st));
  MergeArgs ma;
  ma.db64 = nullptr;
  ma.rec = x->rec.as<float4>();
  ma.recT = x->recT.as<float>();
  ma.q64 = nullptr;
  ma.qn2 = x->qn2.as<double>();
  ma.Rbits = x->Rbits.as<unsigned>();
  ma.nwg = x->nwg;
  ma.tpw = x->tpw;
  ma.pos0 = 0;
  ma.pos_end = x->n_tiles * IA_TILE;
  ma.NT = x->n_tiles;
  ma.NA = (int)x->n;
  ma.pos2row = nullptr;
  ma.rr = 0;
  ma.qinfo = nullptr;
  ma.boxes = nullptr;
  ma.ufac = 0.;
  ma.img_rows = 0;
  ma.eps_c = ia_eps_c(DP);
  ma.eps_a = 0.;
  const int qtmax = ia_k3_qtmax(x->KH);
  for (int64_t b0 = 0; b0 < nq; b0 += BATCH) {
    const int64_t nb = std::min(BATCH, nq - b0);
    const int Mpad = (int)((nb + IA_TILE - 1) / IA_TILE * IA_TILE);
    HIP_TRY(hipMemcpyAsync(x->q.p, q + b0 * x->d, (size_t)nb * x->d * 8, hipMemcpyHostToDevice, c->st));
    ia_launch_dense_query(x->KH, x->q.as<double>(), nb, x->d, Mpad, x->mu.as<double>(), x->qn2.as<double>(),
                          x->qf.as<float>(), c->st);
    const int qtt = Mpad / IA_TILE;
    for (int qt0 = 0; qt0 < qtt; qt0 += qtmax) {
      const int qt = std::min(qtmax, qtt - qt0);
      ia_launch_k3(x->KH, qt, x->db.as<float4>(), x->qf.as<float4>(), x->n_tiles, x->tpw, qt0, (int)nb, x->nwg, 0, x->n_tiles,
                   x->rec.as<float4>(), x->recT.as<float>(), c->st);
    }
    ia_launch_merge_dense(ma, x->pts.as<double>(), x->d, x->q.as<double>(), nb, x->idx.as<int64_t>(),
                          x->dist.as<double>(), c->st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(idx_out + b0, x->idx.p, (size_t)nb * 8, hipMemcpyDeviceToHost, c->st));
    if (dist_out) HIP_TRY(hipMemcpyAsync(dist_out + b0, x->dist.p, (size_t)nb * 8, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
  }
  return IA_OK;
}

int ia_coherence_batch(ia_index *x, const double *q, int64_t nq, const int32_t *px, const int32_t *s, const int32_t *im,
                       int64_t n_s, int a_h, int a_w, int bp_w, int pad, int32_t *p_out, int32_t *img_out, int32_t *rstar_out) {
  if (!x || nq < 0 || n_s < 0 || a_h < 1 || a_w < 1 || bp_w < 1 || pad < 0 || (pad + 1) * (2 * pad + 1) > 64)
    return fail(IA_EINVAL, "ia_coherence_batch: bad arguments (pad must be 0..4)");
  if (nq == 0) return IA_OK;
  if (!q || !px || !p_out || !img_out || !rstar_out || (n_s > 0 && (!s || !im)))
    return fail(IA_EINVAL, "ia_coherence_batch: NULL buffer");
  ia_ctx *c = x->ctx;
  HIP_TRY(hipSetDevice(c->dev));
  int rc;
  if ((rc = x->q.ensure((size_t)nq * x->d * 8)) || (rc = x->cpx.ensure((size_t)nq * 8)) ||
      (rc = x->cs.ensure((size_t)std::max<int64_t>(n_s, 1) * 8)) || (rc = x->cim.ensure((size_t)std::max<int64_t>(n_s, 1) * 4)) ||
      (rc = x->cout.ensure((size_t)nq * 20 + 16)))
    return rc;
  int32_t *dp = x->cout.as<int32_t>(), *di = dp + 2 * nq, *dr = di + nq;
  unsigned *derr = reinterpret_cast<unsigned *>(dr + 2 * nq);
  HIP_TRY(hipMemcpyAsync(x->q.p, q, (size_t)nq * x->d * 8, hipMemcpyHostToDevice, c->st));
  HIP_TRY(hipMemcpyAsync(x->cpx.p, px, (size_t)nq * 8, hipMemcpyHostToDevice, c->st));
  if (n_s > 0) {
    HIP_TRY(hipMemcpyAsync(x->cs.p, s, (size_t)n_s * 8, hipMemcpyHostToDevice, c->st));
    HIP_TRY(hipMemcpyAsync(x->cim.p, im, (size_t)n_s * 4, hipMemcpyHostToDevice, c->st));
  }
  HIP_TRY(hipMemsetAsync(derr, 0, 4, c->st));
  ia_launch_coherence_batch(x->pts.as<double>(), x->n, x->d, x->q.as<double>(), nq, x->cpx.as<int32_t>(), x->cs.as<int32_t>(),
                            x->cim.as<int32_t>(), n_s, a_h, a_w, bp_w, pad, dp, di, dr, derr, c->st);
  HIP_TRY(hipGetLastError());
  unsigned err = 0;
  HIP_TRY(hipMemcpyAsync(p_out, dp, (size_t)nq * 8, hipMemcpyDeviceToHost, c->st));
  HIP_TRY(hipMemcpyAsync(img_out, di, (size_t)nq * 4, hipMemcpyDeviceToHost, c->st));
  HIP_TRY(hipMemcpyAsync(rstar_out, dr, (size_t)nq * 8, hipMemcpyDeviceToHost, c->st));
  HIP_TRY(hipMemcpyAsync(&err, derr, 4, hipMemcpyDeviceToHost, c->st));
  HIP_TRY(hipStreamSynchronize(c->st));
  if (err & 1u) return fail(IA_EINVAL, "ia_coherence_batch: a causal neighbour lies beyond the n_s entries of s / im");
  if (err & 2u) return fail(IA_EINVAL, "ia_coherence_batch: a coherence candidate's DB row lies beyond the index");
  return IA_OK;
}

void ia_index_destroy(ia_index *x) {
  if (!x) return;
  hipSetDevice(x->ctx->dev);
  hipStreamSynchronize(x->ctx->st);
  for (DevBuf *b : {&x->pts, &x->db, &x->mu, &x->Rbits, &x->q, &x->q64, &x->qn2, &x->qf, &x->rec, &x->recT, &x->idx,
                    &x->dist, &x->counters, &x->cpx, &x->cs, &x->cim, &x->cout})
    b->release();
  delete x;
}

}  // extern "C"
