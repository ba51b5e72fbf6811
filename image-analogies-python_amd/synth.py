"""Synthetic A / A' / B workloads of the sizes BASELINE.json names.

There is no network and the reference's own input images are not in its repository, so every
benchmark and scale test runs on these generators (legacy MT19937 RandomState, deterministic):
    A  = smooth(h, w, sigma=2, seed=1)        smooth = normalise01(gaussian_filter(rand, sigma))
    A' = clip(A**2.2 + 0.5*(A - gaussian_filter(A, 2)), 0, 1)      tone curve + unsharp mask
    B  = smooth(h, w, sigma=2, seed=2)
    B' init: initialize_Bp(..., init_rand=True, seed=3)
"""
import numpy as np
from scipy.ndimage import gaussian_filter

from . import config as _config
from .img_preprocess import compute_gaussian_pyramid, initialize_Bp


def smooth(h, w, sigma, seed, ch=None):
    rs = np.random.RandomState(seed)
    if ch is None:
        x = gaussian_filter(rs.rand(h, w), sigma)
    else:
        x = np.dstack([gaussian_filter(rs.rand(h, w), sigma) for _ in range(ch)])
    x = x - x.min()
    return x / x.max()


def filt(A):
    s = (2, 2, 0) if A.ndim == 3 else 2
    return np.clip(A ** 2.2 + 0.5 * (A - gaussian_filter(A, s)), 0, 1)


class Job(object):
    """Pyramids + parameters of one synthesis job (everything image_analogies_main derives
    before its level loop, image_analogies.py:103-123), aligned coarsest-first."""

    def __init__(self, A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, k, weights):
        self.A_pyr, self.Ap_pyr_list, self.B_pyr, self.Bp_init = A_pyr, Ap_pyr_list, B_pyr, Bp_pyr
        self.k = k
        self.weights = weights
        self.L = min(len(A_pyr), len(B_pyr))

    def kappa_factor(self, level):
        return 1 + (2 ** (level - self.L)) * self.k   # image_analogies.py:206

    @property
    def pixels(self):
        """B' pixels synthesised by one run (levels 1 .. L-1)."""
        return int(sum(np.prod(self.B_pyr[l].shape[:2]) for l in range(1, self.L)))

    def flops(self):
        """Algorithmic NN flops of one run: sum_l 2 * D * N_A,l * N_B,l."""
        ch = 1 if self.A_pyr[0].ndim == 2 else self.A_pyr[0].shape[2]
        D = 55 * ch
        nap = len(self.Ap_pyr_list)
        return float(sum(2.0 * D * nap * np.prod(self.A_pyr[l].shape[:2]) * np.prod(self.B_pyr[l].shape[:2])
                         for l in range(1, self.L)))


def make_job(size=1024, b_size=None, n_levels=None, k=0.5, seed_a=1, seed_b=2, seed_bp=3, level_align='coarse'):
    """A/A'/B synthetic job.  size: A (and default B) side; n_levels caps the pyramid depth
    (cfg2 uses 5); the pyramid rule otherwise is the reference's (min_size = n_sm = 3).
    level_align: 'coarse' = the reference's alignment of unequal pyramids (coarsest levels
    paired, B's extra fine levels dropped, image_analogies.py:82-86); 'fine' = B's finest level
    paired with A's finest (B level k + d <-> A level k; config.level_align, cfg4)."""
    ah, aw = (size, size) if np.isscalar(size) else size
    b_size = (ah, aw) if b_size is None else b_size
    bh, bw = (b_size, b_size) if np.isscalar(b_size) else b_size
    A = smooth(ah, aw, 2, seed_a)
    Ap = filt(A)
    B = smooth(bh, bw, 2, seed_b)
    A_pyr = compute_gaussian_pyramid(A, _config.n_sm, n_levels)
    Ap_pyr = compute_gaussian_pyramid(Ap, _config.n_sm, n_levels)
    B_pyr = compute_gaussian_pyramid(B, _config.n_sm, n_levels)
    L = min(len(A_pyr), len(B_pyr))
    # the deeper pyramid drops its extra coarse levels ('fine': finest levels paired, as
    # sweep.Sweep / config.level_align) or its extra fine levels ('coarse', the reference)
    sl = slice(-L, None) if level_align == 'fine' else slice(None, L)
    A_pyr, Ap_pyr, B_pyr = A_pyr[sl], Ap_pyr[sl], B_pyr[sl]
    Bp = initialize_Bp(B_pyr, init_rand=True, seed=seed_bp)
    weights = _config.compute_weights(_config.n_sm, _config.n_lg, _config.n_half, 1)
    return Job(A_pyr, [Ap_pyr], B_pyr, Bp, k, weights)


def make_jobs(n, **kw):
    """n jobs of make_job(**kw) that share the A side (the same A / A' pyramid arrays: one
    feature DB per level for all of them, ia_synthesize_levels) with different B images and B'
    inits: job 0 is make_job(**kw) itself, job j > 0 draws B with seed_b + 100 j and B' with
    seed_bp + 100 j (e.g. frames of one video through the same filter)."""
    j0 = make_job(**kw)
    out = [j0]
    for j in range(1, n):
        bh, bw = j0.B_pyr[-1].shape[:2]
        B = smooth(bh, bw, 2, kw.get('seed_b', 2) + 100 * j)
        B_pyr = compute_gaussian_pyramid(B, _config.n_sm, kw.get('n_levels'))
        B_pyr = B_pyr[len(B_pyr) - j0.L:] if kw.get('level_align', 'coarse') == 'fine' else B_pyr[:j0.L]
        Bp = initialize_Bp(B_pyr, init_rand=True, seed=kw.get('seed_bp', 3) + 100 * j)
        out.append(Job(j0.A_pyr, j0.Ap_pyr_list, B_pyr, Bp, j0.k, j0.weights))
    return out


CONFIGS = {
    # name: (kwargs, description) — BASELINE.json configs
    'cfg1': (dict(size=(117, 180)), "shore-crop stand-in 117x180 (CPU reference path config)"),
    'cfg2': (dict(size=512, n_levels=5), "512x512 synthetic A/A'/B, 5-level pyramid, 1 GPU"),
    'cfg3': (dict(size=1024), "1024x1024 synthetic A/A'/B, full 10-level pyramid"),
    'cfg4': (dict(size=1024, b_size=2048, k=25.0, level_align='fine'),
             "2048x2048 B against 1024x1024 A/A' (Freud-crop-style filter), kappa 25, B's finest level paired "
             "with A's (level_align='fine')"),
    'cfg5': (dict(size=512), "multi_script-style sweep: 64 jobs, kappa {0.5,1,2,5,10,15,20,25} x pyramid "
                             "depth 2..9 on 512x512 A/A'/B, job j on GPU j mod N, jobs sharing a GPU batched"),
    'small': (dict(size=128), "128x128 smoke size"),
    's256': (dict(size=256), "256x256 synthetic A/A'/B (multi-rank parity tests)"),
}
