"""CPU restatement (numpy, fp64) of the reference's per-level best-match synthesis path.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import this module, and only as the checker / the timed CPU baseline.  The product
(image-analogies-python_amd/) never imports it and has no CPU fallback.

Pinned against the golden vectors in tests/golden/ that oracle/gen_golden.py produced by
running the real reference (lib2to3 copy + exact-linear pyflann stand-in) in the build
container: feature layout, DB rows, per-pixel NN index, coherence result, weighted distances,
final B' levels and source maps s / im (tests/test_oracle_golden.py).

Every function cites the reference line it restates.  Arithmetic that decides an argmin is
kept bit-identical to the reference's numpy expressions:
  * NN distance: ((As - q)**2).sum(axis=1)  -> numpy pairwise summation (stand-in FLANN linear)
  * coherence:   norm(As[prs] - q, ord=2, axis=1) = sqrt(add.reduce(x*x, axis=1))  (algorithms.py:126)
  * kappa test:  norm((a-q)*w, ord=2)**2 (algorithms.py:135), compared exactly as image_analogies.py:206
"""
import math
import time

import numpy as np

N_SM, N_LG, N_HALF = 3, 5, 12          # config.py:15-18 (n_half as int)


# ----------------------------------------------------------------------------- reference helpers
def reflect(i, n):
    """np.pad(mode='symmetric') index map (img_preprocess.py:81-83), valid for any pad width."""
    i = np.asarray(i) % (2 * n)
    return np.where(i >= n, 2 * n - 1 - i, i)


def matlab_style_gauss2D(shape, sigma):
    """config.py:52-65."""
    m, n = [(ss - 1.) / 2. for ss in shape]
    y, x = np.ogrid[-m:m + 1, -n:n + 1]
    h = np.exp(-(x * x + y * y) / (2. * sigma * sigma))
    h[h < np.finfo(h.dtype).eps * h.max()] = 0
    s = h.sum()
    if s != 0:
        h /= s
    return h


def compute_weights(num_ch):
    """config.py:68-79: [w_sm, w_lg, w_sm, w_half], channel-minor interleave."""
    g_sm = np.repeat(matlab_style_gauss2D((N_SM, N_SM), 0.5).ravel(), num_ch)
    g_lg = np.repeat(matlab_style_gauss2D((N_LG, N_LG), 1).ravel(), num_ch)
    w_sm = (1. / (N_SM * N_SM)) * g_sm
    w_lg = (1. / (N_LG * N_LG)) * g_lg
    w_half = (1. / N_HALF) * g_lg[:N_HALF * num_ch]
    return np.hstack([w_sm, w_lg, w_sm, w_half])


def nch(img):
    return 1 if img.ndim == 2 else img.shape[2]


def _chv(img):
    return img if img.ndim == 3 else img[:, :, None]


def coarse_patch(sm, r, c):
    """3x3 patch of the symmetric-padded coarse level at (floor(r/2), floor(c/2)), flattened
    row-major / channel-minor (algorithms.py:23,39 and :81-82).  r, c: int arrays."""
    s = _chv(sm)
    h, w = s.shape[:2]
    rr = reflect((r // 2)[:, None] + np.arange(-1, 2)[None, :], h)       # (n,3)
    cc = reflect((c // 2)[:, None] + np.arange(-1, 2)[None, :], w)
    p = s[rr[:, :, None], cc[:, None, :]]                                 # (n,3,3,ch)
    return p.reshape(len(r), -1)


def fine_patch(lg, r, c, half):
    """5x5 patch of the symmetric-padded fine level at (r, c), flattened row-major /
    channel-minor, truncated to the first n_half*ch values when `half` (algorithms.py:24,31,83-89)."""
    s = _chv(lg)
    h, w = s.shape[:2]
    rr = reflect(r[:, None] + np.arange(-2, 3)[None, :], h)
    cc = reflect(c[:, None] + np.arange(-2, 3)[None, :], w)
    p = s[rr[:, :, None], cc[:, None, :]].reshape(len(r), -1)
    return p[:, :N_HALF * s.shape[2]] if half else p


def feature_array(pyr, level, full):
    """compute_feature_array (algorithms.py:11-47) for one level >= 1 (raster order rows)."""
    h, w = pyr[level].shape[:2]
    assert pyr[level - 1].shape[0] == -(-h // 2) and pyr[level - 1].shape[1] == -(-w // 2)
    r, c = np.divmod(np.arange(h * w), w)
    return np.hstack([coarse_patch(pyr[level - 1], r, c), fine_patch(pyr[level], r, c, not full)])


def build_db(A_pyr, Ap_pyr_list, level):
    """create_index's As[level] (algorithms.py:50-70): vstack_i hstack(A_full, A'_i_half)."""
    Af = feature_array(A_pyr, level, True)
    return np.vstack([np.hstack([Af, feature_array(p, level, False)]) for p in Ap_pyr_list])


def query_feature(B_feat_l, Bp_sm, Bp_lg, r, c, w):
    """BBp_feat (image_analogies.py:166-168 + algorithms.py:78-89) for pixel (r, c)."""
    ra, ca = np.array([r]), np.array([c])
    return np.hstack([B_feat_l[r * w + c], coarse_patch(Bp_sm, ra, ca)[0], fine_patch(Bp_lg, ra, ca, True)[0]])


def nn_exact(As, q):
    """best_approximate_match (algorithms.py:73-75) with FLANN-linear semantics: fp64 squared
    L2 with numpy's pairwise summation, first (lowest-index) argmin."""
    d = ((As - q) ** 2).sum(axis=1)
    i = int(np.argmin(d))
    return i, d


def coherence(As, A_h, A_w, q, s, im, r, c, w):
    """best_coherence_match (algorithms.py:92-130).  s: (N,2) int array, im: (N,) int array,
    valid for raster indices < r*w+c.  Returns ((pr, pc), img, (rr, rc)) or ((-1,-1), 0, (0,0))."""
    cand, src = [], []
    qi = r * w + c
    for rr in range(max(0, r - 2), r + 1):
        for rc in range(max(0, c - 2), min(w, c + 3)):
            ri = rr * w + rc
            if ri >= qi:
                continue
            pr, pc = s[ri, 0] + r - rr, s[ri, 1] + c - rc
            if 0 <= pr < A_h and 0 <= pc < A_w:
                cand.append(((A_h * im[ri] + pr) * A_w + pc))
                src.append(((pr, pc), int(im[ri]), (rr, rc)))
    if not cand:
        return (-1, -1), 0, (0, 0)
    x = As[np.array(cand)] - q
    k = int(np.argmin(np.sqrt(np.add.reduce(x * x, axis=1))))
    return src[k]


def compute_distance(a, q, weights):
    """algorithms.py:133-135."""
    return np.linalg.norm((a - q) * weights, ord=2) ** 2


def _fma(a, b, c):
    from fractions import Fraction
    return float(Fraction(a) * Fraction(b) + Fraction(c))   # one rounding, like a hardware FMA


def blas_ddot_sq(x):
    """x.dot(x) in the order of the BLAS behind numpy on the host that made the golden vectors
    (OpenBLAS 0.3.29 ddot, SkylakeX kernel; matched bit-for-bit against np.dot for n = 1..165).
    np.linalg.norm(v, ord=2) of a 1-D v is sqrt(v.dot(v)), so compute_distance's last bits
    depend on this order; the GPU's blas_dot_sq (ia_kernels.hip) restates it.  Pure Python,
    exact FMA via fractions: test-sized inputs only."""
    x = [float(v) for v in x]
    n = len(x)
    n1 = n & ~15
    n32 = n1 & ~31
    z = [[0.0] * 8 for _ in range(4)]
    i = 0
    while i < n32:
        for k in range(4):
            for l in range(8):
                v = x[i + 8 * k + l]
                z[k][l] = _fma(v, v, z[k][l])
        i += 32
    acc = [[z[k][l] + z[k][l + 4] for l in range(4)] for k in range(4)]
    while i < n1:
        for k in range(4):
            for l in range(4):
                v = x[i + 4 * k + l]
                acc[k][l] = _fma(v, v, acc[k][l])
        i += 16
    sl = [((acc[0][l] + acc[1][l]) + acc[2][l]) + acc[3][l] for l in range(4)]
    dot = (sl[0] + sl[2]) + (sl[1] + sl[3]) if n1 else 0.0
    for j in range(n1, n):
        dot = _fma(x[j], x[j], dot)
    return dot


def compute_distance_blas(a, q, weights):
    """compute_distance with the dot order made explicit (blas_ddot_sq), machine-independent."""
    return np.sqrt(blas_ddot_sq((a - q) * weights)) ** 2


# ----------------------------------------------------------------------------- the level loop
def synthesize_level(A_pyr, Ap_pyr_list, B_feat_l, Bp_pyr, level, L, k, weights,
                     As=None, faithful_pad=False, max_pixels=None, log=None, start_pixel=0, s_state=None,
                     im_state=None):
    """One level of image_analogies_main's raster loop (image_analogies.py:130-239).

    Bp_pyr[level] is updated in place (as the reference does).  Returns s (N,2), im (N,).
    faithful_pad: re-pad the B' pair on every pixel like image_analogies.py:166 (CPU-baseline
    cost model); the decisions are identical either way.
    max_pixels: stop after that many raster pixels (bounded CPU-baseline sample).
    start_pixel, s_state, im_state: resume at raster pixel start_pixel of a level whose earlier
    pixels are already synthesised (Bp_pyr[level] and s_state / im_state hold them, e.g. a GPU
    run's final state; bench.py's mid-level CPU-baseline sample)."""
    if As is None:
        As = build_db(A_pyr, Ap_pyr_list, level)
    h, w = Bp_pyr[level].shape[:2]
    A_h, A_w = Ap_pyr_list[0][level].shape[:2]
    n = h * w if max_pixels is None else min(h * w, start_pixel + max_pixels)
    s = np.zeros((h * w, 2), dtype=np.int64) if s_state is None else np.array(s_state, dtype=np.int64)
    im = np.zeros(h * w, dtype=np.int64) if im_state is None else np.array(im_state, dtype=np.int64)
    kf = 1 + (2 ** (level - L)) * k
    ch = nch(Bp_pyr[level])
    for qi in range(start_pixel, n):
        r, c = divmod(qi, w)
        if faithful_pad:
            p1 = ((1, 1), (1, 1)) + (((0, 0),) if ch > 1 else ())
            p2 = ((2, 2), (2, 2)) + (((0, 0),) if ch > 1 else ())
            sm_pd = np.pad(Bp_pyr[level - 1], p1, mode='symmetric')
            lg_pd = np.pad(Bp_pyr[level], p2, mode='symmetric')
            q = np.hstack([B_feat_l[qi], sm_pd[r // 2:r // 2 + 3, c // 2:c // 2 + 3].ravel(),
                           lg_pd[r:r + 5, c:c + 5].ravel()[:N_HALF * ch]])
        else:
            q = query_feature(B_feat_l, Bp_pyr[level - 1], Bp_pyr[level], r, c, w)
        p_ix, _ = nn_exact(As, q)
        i_app, rem = divmod(p_ix, A_h * A_w)
        p_app = divmod(rem, A_w)
        p, i = p_app, i_app
        rec = None
        if qi > 0:
            p_coh, i_coh, r_star = coherence(As, A_h, A_w, q, s, im, r, c, w)
            if p_coh != (-1, -1):
                d_app = compute_distance(As[p_ix], q, weights)
                d_coh = compute_distance(As[(A_h * i_coh + p_coh[0]) * A_w + p_coh[1]], q, weights)
                if d_coh <= d_app * kf:
                    p, i = p_coh, i_coh
                rec = (p_coh, i_coh, d_app, d_coh)
        if log is not None:
            log.append((p_ix, rec))
        Bp_pyr[level][r, c] = Ap_pyr_list[i][level][p]
        s[qi] = p
        im[qi] = i
    return s, im


def run_all_levels(A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, k, weights, log=None, faithful_pad=False):
    """image_analogies_main's level loop (image_analogies.py:111,119,130): levels 1..L-1,
    L = number of pyramid images (both pyramids aligned coarsest-first, :82-86)."""
    L = min(len(A_pyr), len(B_pyr))
    S, IM = {}, {}
    for level in range(1, L):
        B_feat = feature_array(B_pyr, level, True)
        S[level], IM[level] = synthesize_level(A_pyr, Ap_pyr_list, B_feat, Bp_pyr, level, L, k,
                                               weights, log=log, faithful_pad=faithful_pad)
    return S, IM


# ----------------------------------------------------------------------------- teacher forcing
def state_at(final, init, qi):
    """B' level as the raster loop saw it while deciding raster pixel qi: pixels before qi hold
    their final (synthesised) value, the rest still hold the initial value."""
    h, w = final.shape[:2]
    m = (np.arange(h * w) < qi).reshape(h, w)
    if final.ndim == 3:
        m = m[:, :, None]
    return np.where(m, final, init)


def decide_pixel(As, B_feat_l, Bp_sm, Bp_final, Bp_init, s, im, A_h, A_w, level, L, k,
                 weights, r, c):
    """Re-decide raster pixel (r, c) with the reference's decision functions on a build's state
    (SURVEY §7 hard part 2).  Returns a dict with the oracle's choice and its margins."""
    h, w = Bp_final.shape[:2]
    qi = r * w + c
    lg = state_at(Bp_final, Bp_init, qi)
    q = query_feature(B_feat_l, Bp_sm, lg, r, c, w)
    p_ix, d = nn_exact(As, q)
    d_sorted = np.partition(d, 1)[:2] if len(d) > 1 else np.array([d[0], np.inf])
    out = {'q': q, 'app_ix': p_ix, 'app_d': d[p_ix], 'app_gap': (d_sorted[1] - d_sorted[0]) / max(d_sorted[0], 1e-300),
           'choice': None, 'coh': None}
    i_app, rem = divmod(p_ix, A_h * A_w)
    p_app = divmod(rem, A_w)
    out['choice'] = (p_app, i_app)
    if qi > 0:
        p_coh, i_coh, _ = coherence(As, A_h, A_w, q, s, im, r, c, w)
        out['coh'] = (p_coh, i_coh)
        if p_coh != (-1, -1):
            d_app = compute_distance(As[p_ix], q, weights)
            d_coh = compute_distance(As[(A_h * i_coh + p_coh[0]) * A_w + p_coh[1]], q, weights)
            kf = 1 + (2 ** (level - L)) * k
            out['d_app'], out['d_coh'] = d_app, d_coh
            out['kappa_gap'] = abs(d_coh - d_app * kf) / max(d_app * kf, 1e-300)
            if d_coh <= d_app * kf:
                out['choice'] = (p_coh, i_coh)
    return out


# ----------------------------------------------------------------------------- CPU baseline
def time_sample(A_pyr, Ap_pyr_list, B_pyr, Bp_pyr, level, L, k, weights, n_pixels, start=0, state=None,
                As=None, B_feat=None):
    """Time the reference loop (faithful per-pixel pad, exact fp64 NN) on n_pixels consecutive
    raster pixels of `level` from raster pixel `start`; returns seconds per pixel (SURVEY §8(d)
    CPU-baseline plan).  state = (Bp level, s, im) of an already synthesised level (a mid-level
    sample resumes on it); As / B_feat may be passed in (shared by several sampling threads)."""
    B_feat = feature_array(B_pyr, level, True) if B_feat is None else B_feat
    As = build_db(A_pyr, Ap_pyr_list, level) if As is None else As
    Bp = [x.copy() for x in Bp_pyr]
    s0 = im0 = None
    if state is not None:
        Bp[level] = np.array(state[0], dtype=np.float64).reshape(Bp[level].shape)
        s0, im0 = state[1], state[2]
    t0 = time.perf_counter()
    synthesize_level(A_pyr, Ap_pyr_list, B_feat, Bp, level, L, k, weights, As=As,
                     faithful_pad=True, max_pixels=n_pixels, start_pixel=start, s_state=s0, im_state=im0)
    return (time.perf_counter() - t0) / n_pixels
