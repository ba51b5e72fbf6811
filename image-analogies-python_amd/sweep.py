"""Parameter sweeps over one A / A' / B triple (multi_script.py, BASELINE config 5).

The reference sweeps by calling image_analogies_main once per setting, mutating the config
module between calls (multi_script.py:13-32: c.k over a kappa list; other scripts vary the
pyramid depth, AB_weight or the A' set).  Every such job re-reads the images, rebuilds every
level's feature DB and runs its own raster loop.  Here the jobs of a sweep that share the A side
run together:

  * the image pyramids are computed once.  A job with n_levels = n uses the finest n levels of
    the full pyramid (pyramid_gaussian stops earlier; the levels it does make are identical);
  * levels are processed resolution by resolution, coarse to fine.  At each resolution every
    job that synthesises a level there joins ONE ia_synthesize_levels call: one DB build, and
    per wavefront step one gather, one distance scan over the DB for all jobs' queries and one
    merge (include/ia.h).  Each job's results are bit-identical to running it alone;
  * on several GPUs, job j runs on rank j mod world (no collective: the jobs are independent).

The kappa factor of a job's level l is 1 + 2^(l - L_j) k_j with L_j its own pyramid depth
(image_analogies.py:206).
"""
import warnings

import numpy as np

from . import _native
from . import config as _config
from .img_preprocess import compute_gaussian_pyramid, initialize_Bp


class SweepJob(object):
    """One job of a sweep: kappa, pyramid depth (None: the reference rule) and B' seed."""

    def __init__(self, k=0.5, n_levels=None, seed=3, init_rand=True):
        self.k, self.n_levels, self.seed, self.init_rand = float(k), n_levels, seed, init_rand

    def __repr__(self):
        return 'SweepJob(k=%g, n_levels=%s, seed=%s)' % (self.k, self.n_levels, self.seed)


def cfg5_jobs(kappas=(0.5, 1, 2, 5, 10, 15, 20, 25), depths=range(2, 10), seed=3):
    """BASELINE config 5: kappa x pyramid depth (64 jobs on 512^2 images), depth-major, so that
    job j -> GPU j mod 8 gives every GPU one job of each depth (balanced work)."""
    return [SweepJob(k, n, seed) for n in depths for k in kappas]


class Sweep(object):
    """Host side of a sweep: the full pyramids of A, A'_i, B and each job's B' pyramid.
    full_levels(j) maps job j's level l to the full pyramid's index f = l + (Lf - L_j)."""

    def __init__(self, A, Ap_list, B, jobs, weights=None, min_size=None, level_align='coarse'):
        """level_align (config.level_align): how pyramids of unequal depth pair up.  'coarse' is
        the reference's rule (image_analogies.py:82-86): the coarsest levels pair and the deeper
        pyramid's extra fine levels are dropped, with the reference's warning; 'fine' pairs the
        finest levels (B level k + d <-> A level k, cfg4's pairing)."""
        min_size = _config.n_sm if min_size is None else min_size
        if level_align not in ('coarse', 'fine'):
            raise ValueError("level_align must be 'coarse' or 'fine'")
        self.A_pyr = compute_gaussian_pyramid(A, min_size)
        self.Ap_pyr_list = [compute_gaussian_pyramid(Ap, min_size) for Ap in Ap_list]
        self.B_pyr = compute_gaussian_pyramid(B, min_size)
        Lf = min(len(self.A_pyr), len(self.B_pyr))
        if len(self.A_pyr) != len(self.B_pyr):
            warnings.warn('Warning: input images are very different sizes! The minimum number of levels will be used.')
        sl = slice(None, Lf) if level_align == 'coarse' else slice(-Lf, None)
        self.A_pyr, self.B_pyr = self.A_pyr[sl], self.B_pyr[sl]
        self.Ap_pyr_list = [p[sl] for p in self.Ap_pyr_list]
        for a, b in zip(self.A_pyr, self.B_pyr):   # paired levels: same depth below the coarsest
            assert a.ndim == b.ndim, 'A and B differ in channels'
        self.Lf = Lf
        ch = 1 if A.ndim == 2 else A.shape[2]
        self.weights = (_config.compute_weights(_config.n_sm, _config.n_lg, _config.n_half, ch)
                        if weights is None else weights)
        self.jobs = list(jobs)
        self.L = [min(Lf, j.n_levels) if j.n_levels else Lf for j in self.jobs]
        self.Bp_init = [initialize_Bp(self.B_pyr[Lf - L:], init_rand=j.init_rand, seed=j.seed)
                        for j, L in zip(self.jobs, self.L)]

    def offset(self, j):
        return self.Lf - self.L[j]

    def kappa_factor(self, j, level):
        return 1 + (2 ** (level - self.L[j])) * self.jobs[j].k    # image_analogies.py:206

    def pixels(self, jobs=None):
        """B' pixels synthesised by the given jobs (levels 1 .. L_j - 1 of each)."""
        jobs = range(len(self.jobs)) if jobs is None else jobs
        return int(sum(np.prod(self.B_pyr[self.offset(j) + l].shape[:2]) for j in jobs for l in range(1, self.L[j])))

    def schedule(self, jobs=None, max_batch=16):
        """[(f, [(job, level), ...]), ...]: per full-pyramid level f (coarse to fine) the jobs that
        synthesise a level there, in batches of at most max_batch."""
        jobs = range(len(self.jobs)) if jobs is None else jobs
        out = []
        for f in range(1, self.Lf):
            part = [(j, f - self.offset(j)) for j in jobs if f - self.offset(j) >= 1]
            for b in range(0, len(part), max_batch):
                out.append((f, part[b:b + max_batch]))
        return out

    def run(self, ctx, jobs=None, batched=True, max_batch=16, stats=None):
        """Synthesise the given jobs (default: all) on ctx with host buffers.  batched=False runs
        every job level by level on its own (the reference's one-job-at-a-time sweep).
        Returns {job: (Bp_pyr, {level: s}, {level: im})}."""
        jobs = list(range(len(self.jobs)) if jobs is None else jobs)
        Bp = {j: [x.copy() for x in self.Bp_init[j]] for j in jobs}
        S = {j: {} for j in jobs}
        IM = {j: {} for j in jobs}
        stats = stats if stats is not None else _native.Stats()
        for f, part in self.schedule(jobs, max_batch if batched else 1):
            A, Ac = self.A_pyr[f], self.A_pyr[f - 1]
            Ap = [p[f] for p in self.Ap_pyr_list]
            Apc = [p[f - 1] for p in self.Ap_pyr_list]
            specs = [dict(B=self.B_pyr[f], Bc=self.B_pyr[f - 1], Bpc=Bp[j][l - 1], Bp=Bp[j][l], weights=self.weights,
                          kappa_factor=self.kappa_factor(j, l)) for j, l in part]
            res = ctx.synthesize_levels(A, Ac, Ap, Apc, specs, stats)
            for (j, l), (s, im) in zip(part, res):
                S[j][l], IM[j][l] = s, im
        return {j: (Bp[j], S[j], IM[j]) for j in jobs}


class DeviceSweep(object):
    """A sweep with every input resident in HBM (torch tensors; bench.py --config cfg5): the full
    pyramids once, each job's B' pyramid and source maps.  run() re-initialises B' on the device
    and synthesises the jobs; nothing crosses PCIe inside it."""

    def __init__(self, sweep, jobs, torch, dev):
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).to(dev)
        self.sw, self.jobs, self.torch = sweep, list(jobs), torch
        self.A = [t(x) for x in sweep.A_pyr]
        self.Ap = [t(np.stack([p[f] for p in sweep.Ap_pyr_list])) for f in range(sweep.Lf)]
        self.B = [t(x) for x in sweep.B_pyr]
        self.W = t(sweep.weights)
        self.Bp0 = {j: [t(x) for x in sweep.Bp_init[j]] for j in self.jobs}
        self.Bp = {j: [x.clone() for x in self.Bp0[j]] for j in self.jobs}
        hw = lambda x: int(np.prod(x.shape[:2]))
        self.S = {j: [torch.empty((hw(x), 2), dtype=torch.int32, device=dev) for x in self.Bp0[j]] for j in self.jobs}
        self.IM = {j: [torch.empty(hw(x), dtype=torch.int32, device=dev) for x in self.Bp0[j]] for j in self.jobs}
        self.ch = 1 if sweep.A_pyr[0].ndim == 2 else sweep.A_pyr[0].shape[2]

    def run(self, ctx, stats, batched=True, max_batch=16):
        """ctx: one libia Context, or a list of them: the jobs are then dealt round-robin over the
        contexts (each with its own HIP stream) and synthesised by one host thread per context, so
        one group's latency-bound merge / gather kernels overlap another group's scans (libia's
        calls release the GIL; per-thread stats are summed into `stats`)."""
        for j in self.jobs:
            for a, b in zip(self.Bp[j], self.Bp0[j]):
                a.copy_(b)
        self.torch.cuda.synchronize()   # libia runs on its own stream(s)
        if isinstance(ctx, (list, tuple)) and len(ctx) > 1:
            import threading
            from . import _native
            groups = [self.jobs[i::len(ctx)] for i in range(len(ctx))]
            sts = [_native.Stats() for _ in ctx]
            errs = []

            def work(c, jobs, st):
                try:
                    self._run_jobs(c, jobs, st, batched, max_batch)
                except Exception as e:  # re-raised on the calling thread
                    errs.append(e)
            th = [threading.Thread(target=work, args=(c, g, st)) for c, g, st in zip(ctx, groups, sts)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            if errs:
                raise errs[0]
            for st in sts:
                stats.add(st)
            return
        self._run_jobs(ctx[0] if isinstance(ctx, (list, tuple)) else ctx, self.jobs, stats, batched, max_batch)

    def _run_jobs(self, ctx, jobs, stats, batched, max_batch):
        sw = self.sw
        for f, part in sw.schedule(jobs, max_batch if batched else 1):
            ptrs = [dict(A=self.A[f].data_ptr(), Ac=self.A[f - 1].data_ptr(), Ap=self.Ap[f].data_ptr(),
                         Apc=self.Ap[f - 1].data_ptr(), B=self.B[f].data_ptr(), Bc=self.B[f - 1].data_ptr(),
                         Bpc=self.Bp[j][l - 1].data_ptr(), Bp=self.Bp[j][l].data_ptr(), weights=self.W.data_ptr(),
                         s_out=self.S[j][l].data_ptr(), im_out=self.IM[j][l].data_ptr()) for j, l in part]
            kfs = [sw.kappa_factor(j, l) for j, l in part]
            ctx.synthesize_levels_device(self.ch, len(sw.Ap_pyr_list), self.A[f].shape[:2], self.B[f].shape[:2], ptrs,
                                         kfs, stats)
