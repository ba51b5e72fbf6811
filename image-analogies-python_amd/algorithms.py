"""Matching API of the reference's algorithms.py, same names and signatures.

Hot-path functions run on the GPU:
  * create_index / best_approximate_match: the FLANN object the reference builds per level
    (algorithms.py:56,69,74) is replaced by GpuFLANN, a duck-typed FLANN whose build_index /
    nn_index run libia's exact MFMA + certified-fp64 1-NN (ia_index_*).  The reference asks
    FLANN for a randomised kd-forest ('kdtree'); every `algorithm` is answered exactly here
    (FLANN `linear` semantics: squared L2, lowest index on ties).
  * image_analogies_main does not call the per-pixel functions at all: the whole level (DB
    build, wavefront, NN, coherence, kappa rule, writeback) is one ia_synthesize_level call.

  * best_coherence_match: libia's ia_coherence_batch (one wave per pixel) against the rows of
    the index create_index built for that level (As[level] carries it, IndexedRows);
    best_coherence_match_batch answers many pixels in one call.

compute_feature_array, extract_pixel_feature and compute_distance are kept as the reference's
per-pixel/array helpers (host numpy over the caller's arrays) for code written against that API;
the level path computes the same quantities on the GPU (K1/K2/K4 in csrc/ia_kernels.hip).
"""
import numpy as np

from . import _native
from .img_preprocess import Ap_px2ix

_CTX = None


def default_context():
    """Process-wide GPU context (device = config.device, LOCAL_RANK or 0)."""
    global _CTX
    if _CTX is None:
        from . import config
        _CTX = _native.Context(config.device)
    return _CTX


def _reflect(i, n):
    i = np.asarray(i) % (2 * n)
    return np.where(i >= n, 2 * n - 1 - i, i)


def _windows(img, rows, cols, half_rows):
    """Patches of a symmetric-padded image around (rows, cols): (n, len(half_rows)**2 * ch),
    flattened row-major / channel-minor like sklearn's extract_patches_2d rows."""
    x = img if img.ndim == 3 else img[:, :, None]
    h, w = x.shape[:2]
    rr = _reflect(rows[:, None] + half_rows[None, :], h)
    cc = _reflect(cols[:, None] + half_rows[None, :], w)
    return x[rr[:, :, None], cc[:, None, :]].reshape(len(rows), -1)


def compute_feature_array(im_pyr, c, full_feat):
    """Per-level feature rows (algorithms.py:11-47): level 0 is [], level l >= 1 is
    (h_l * w_l, (9 + 25 or 12) * ch): the 3x3 window of level l-1 around (r//2, c//2) followed
    by the 5x5 window of level l around (r, c) (first n_half*ch values when not full_feat)."""
    feats = [[]]
    n_sm, n_lg = c.n_sm, c.n_lg
    for level in range(1, len(im_pyr)):
        h, w = im_pyr[level].shape[:2]
        r, col = np.divmod(np.arange(h * w), w)
        sm = _windows(im_pyr[level - 1], r // 2, col // 2, np.arange(n_sm) - n_sm // 2)
        lg = _windows(im_pyr[level], r, col, np.arange(n_lg) - n_lg // 2)
        if not full_feat:
            ch = 1 if im_pyr[level].ndim == 2 else im_pyr[level].shape[2]
            lg = lg[:, :ch * int(c.n_half)]
        feats.append(np.hstack([sm, lg]))
    return feats


class GpuFLANN(object):
    """Duck-typed pyflann.FLANN (algorithms.py:56): build_index(pts, algorithm=...) returns a
    params dict with 'checks'; nn_index(q, 1, checks=...) returns (indices, squared distances).
    Backed by libia's exact GPU index; `algorithm` / `checks` are accepted and recorded."""

    def __init__(self, ctx=None):
        self._ctx = ctx
        self._index = None

    def build_index(self, pts, algorithm='kdtree', **kwargs):
        self._index = _native.ExactIndex(self._ctx or default_context(), pts)
        params = {'algorithm': algorithm, 'checks': kwargs.get('checks', 32), 'exact': True}
        return params

    def nn_index(self, qpts, num_neighbors=1, checks=None, **kwargs):
        if self._index is None:
            raise _native.IAError('nn_index called before build_index')
        if num_neighbors != 1:
            raise _native.IAError('GpuFLANN.nn_index: only num_neighbors=1 is supported')
        idx, dist = self._index.query(np.atleast_2d(qpts))
        return idx, dist

    def delete_index(self):
        if self._index is not None:
            self._index.close()
            self._index = None


class IndexedRows(np.ndarray):
    """The As[level] array of create_index (algorithms.py:63-67) with the GPU index built over it
    attached (`.index`, an _native.ExactIndex), so best_coherence_match finds the device copy of
    the rows instead of uploading them per call.  Behaves as the plain ndarray otherwise."""

    def __new__(cls, rows, index):
        obj = np.asarray(rows).view(cls)
        obj.index = index
        return obj

    def __array_finalize__(self, obj):
        self.index = getattr(obj, 'index', None)


def _rows_index(As):
    idx = getattr(As, 'index', None)
    if idx is not None and idx._h and As.shape == (idx.n, idx.d):
        return idx
    # rows without an attached index (e.g. a caller-built As): one GPU upload for this call
    return _native.ExactIndex(default_context(), np.asarray(As))


def create_index(A_pyr, Ap_pyr_list, c):
    """Per-level DB of [A full feature | A'_i half feature] rows stacked over the A' images and
    its (GPU) index (algorithms.py:50-70).  Returns (flann, flann_params, As, As_size)."""
    A_feat = compute_feature_array(A_pyr, c, full_feat=True)
    Ap_feats = [compute_feature_array(p, c, full_feat=False) for p in Ap_pyr_list]
    L = c.max_levels
    flann = [GpuFLANN() for _ in range(L)]
    flann_params = [[] for _ in range(L)]
    As = [[] for _ in range(L)]
    As_size = [[] for _ in range(L)]
    for level in range(1, L):
        As[level] = np.vstack([np.hstack([A_feat[level], f[level]]) for f in Ap_feats])
        As_size[level] = As[level].shape
        flann_params[level] = flann[level].build_index(As[level], algorithm='kdtree')
        As[level] = IndexedRows(As[level], flann[level]._index)
    return flann, flann_params, As, As_size


def best_approximate_match(flann, params, BBp_feat):
    """algorithms.py:73-75 — exact here (see GpuFLANN)."""
    result, dists = flann.nn_index(BBp_feat, 1, checks=params['checks'])
    return result[0]


def extract_pixel_feature(padded_pair, px, c, full_feat):
    """Feature of one pixel from an already padded (coarse, fine) pair (algorithms.py:78-89)."""
    sm_pd, lg_pd = padded_pair
    row, col = int(px[0]), int(px[1])
    k_sm, k_lg = 2 * int(c.pad_sm) + 1, 2 * int(c.pad_lg) + 1
    coarse = sm_pd[row // 2:row // 2 + k_sm, col // 2:col // 2 + k_sm].ravel()
    fine = lg_pd[row:row + k_lg, col:col + k_lg].ravel()
    feat = np.concatenate([coarse, fine])
    if full_feat:
        return feat
    return feat[:c.num_ch * (c.n_sm * c.n_sm + int(c.n_half))]


def best_coherence_match(As, A_hw, BBp_feat, s, im, px, Bp_w, c):
    """Coherence candidate of pixel px (algorithms.py:92-130), on the GPU (ia_coherence_batch):
    over the already synthesised pixels r of the causal L-shaped window (rows px-2..px, cols
    px-2..px+2, raster-earlier), candidate p = s(r) + (px - r) in image im(r) if inside A; first
    argmin of the unweighted L2 distance.  Returns (p, img, r*) or ((-1, -1), 0, (0, 0)).
    s / im are the level's lists so far (raster order), as the reference keeps them."""
    p, img, rs = best_coherence_match_batch(As, A_hw, np.atleast_2d(BBp_feat), s, im, np.array([px]), Bp_w, c)
    if p[0, 0] < 0:
        return (-1, -1), 0, (0, 0)
    return p[0].astype(np.int64), int(img[0]), rs[0].astype(np.int64)


def best_coherence_match_batch(As, A_hw, BBp_feats, s, im, pxs, Bp_w, c):
    """best_coherence_match for many pixels in one GPU call (e.g. one wavefront step: every
    causal neighbour of every pixel must already be in s / im).  Returns int32 arrays
    p (n, 2), img (n,), r_star (n, 2); p = (-1, -1) where there is no candidate."""
    s = np.asarray(s, dtype=np.int32).reshape(-1, 2)
    im = np.asarray(im, dtype=np.int32).reshape(-1)
    return _rows_index(As).coherence(BBp_feats, pxs, s, im, A_hw, Bp_w, int(c.pad_lg))


def compute_distance(AAp_p, BBp_q, weights):
    """Weighted squared distance used by the kappa rule (algorithms.py:133-135)."""
    if not (AAp_p.shape == BBp_q.shape == weights.shape):
        raise ValueError('compute_distance: shape mismatch')
    return np.linalg.norm((AAp_p - BBp_q) * weights, ord=2) ** 2
