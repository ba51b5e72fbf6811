"""GPU parity of the per-pixel matching API against the reference's own picks.

* algorithms.create_index / best_approximate_match (GpuFLANN) and the pyflann drop-in
  flann_mi355x.FLANN on the random 3-level DBs of features.npz, whose 'rand_c*_nn_2' are the
  reference's best_approximate_match picks (oracle/gen_golden.py ran algorithms.py with the
  exact-linear FLANN stand-in), 1 and 3 channels.
* INTEGRATION.md §1 ("minimal" depth): the reference's per-pixel level loop
  (image_analogies.py:130-239) kept as it is, with pyflann replaced and best_coherence_match
  running on the GPU (ia_coherence_batch), reproduces every NN pick (golden 'app_ix'), every
  coherence pick (golden 'coh'), s, im and B' of the g32 / yiq reference runs.
"""
import os
import types

import numpy as np
import pytest

from golden_util import GOLDEN, load_e2e

pytestmark = pytest.mark.gpu


def _cfg(ch, L):
    from ia_amd import config
    return types.SimpleNamespace(n_sm=3, n_lg=5, n_half=12, pad_sm=1, pad_lg=2, max_levels=L, num_ch=ch,
                                 padding_sm=config.setup_vars(np.zeros((4, 4) + ((ch,) if ch > 1 else ())))[1],
                                 padding_lg=config.setup_vars(np.zeros((4, 4) + ((ch,) if ch > 1 else ())))[2])


@pytest.mark.parametrize('ch', [1, 3])
def test_create_index_best_approximate_match_reference_picks(ch):
    from ia_amd import algorithms
    g = np.load(os.path.join(GOLDEN, 'features.npz'))
    tag = 'rand_c%d' % ch
    A = [g['%s_A_%d' % (tag, l)] for l in range(3)]
    Ap = [g['%s_Ap_%d' % (tag, l)] for l in range(3)]
    c = _cfg(ch, 3)
    flann, params, As, As_size = algorithms.create_index(A, [Ap], c)
    for l in (1, 2):
        assert np.array_equal(np.asarray(As[l]), g['%s_As_%d' % (tag, l)])
        assert As_size[l] == g['%s_As_%d' % (tag, l)].shape
    Q, ref = g['%s_Q_2' % tag], g['%s_nn_2' % tag]
    picks = [algorithms.best_approximate_match(flann[2], params[2], q) for q in Q]   # one call per pixel
    assert np.array_equal(picks, ref)
    idx, dist = flann[2].nn_index(Q, 1, checks=params[2]['checks'])                  # one batched call
    assert np.array_equal(idx, ref)
    assert np.array_equal(dist, ((np.asarray(As[2])[ref] - Q) ** 2).sum(axis=1))


@pytest.mark.parametrize('ch', [1, 3])
def test_flann_mi355x_dropin_reference_picks(ch):
    import ia_amd  # noqa: F401
    from ia_amd import flann_mi355x as pf
    g = np.load(os.path.join(GOLDEN, 'features.npz'))
    tag = 'rand_c%d' % ch
    fl = pf.FLANN()
    params = fl.build_index(g['%s_As_2' % tag], algorithm='kdtree')
    assert params['checks'] == 32
    Q = g['%s_Q_2' % tag]
    assert np.array_equal([fl.nn_index(q, 1, checks=params['checks'])[0][0] for q in Q], g['%s_nn_2' % tag])
    fl.delete_index()


def _reference_loop(z, c, flann, params, As, out):
    """image_analogies.py:130-239 as the reference writes it, on the package's per-pixel API."""
    from ia_amd import algorithms as A
    from ia_amd.img_preprocess import Ap_ix2px, Ap_px2ix, pad_img_pair, px2ix
    Bp_pyr = [x.copy() for x in z['Bp_init']]
    B_features = A.compute_feature_array(z['B_pyr'], c, full_feat=True)
    app_ix, coh = [], []
    for level in range(1, c.max_levels):
        imh, imw = Bp_pyr[level].shape[:2]
        s, im = [], []
        Ap_imh, Ap_imw = z['Ap_pyr'][0][level].shape[:2]
        for row in range(imh):
            for col in range(imw):
                px = np.array([row, col])
                Bp_pd = pad_img_pair(Bp_pyr[level - 1], Bp_pyr[level], c)
                BBp_feat = np.hstack([B_features[level][px2ix(px, imw), :],
                                      A.extract_pixel_feature(Bp_pd, px, c, full_feat=False)])
                p_app_ix = A.best_approximate_match(flann[level], params[level], BBp_feat)
                app_ix.append(p_app_ix)
                p_app, i_app = Ap_ix2px(p_app_ix, Ap_imh, Ap_imw)
                if len(s) < 1:
                    p, i = p_app, i_app
                else:
                    p_coh, i_coh, r_star = A.best_coherence_match(As[level], (Ap_imh, Ap_imw), BBp_feat, s, im, px,
                                                                  imw, c)
                    coh.append((p_coh[0], p_coh[1], i_coh))
                    if np.allclose(p_coh, np.array([-1, -1])):
                        p, i = p_app, i_app
                    else:
                        d_app = A.compute_distance(As[level][p_app_ix], BBp_feat, c.weights)
                        d_coh = A.compute_distance(As[level][Ap_px2ix(p_coh, i_coh, Ap_imh, Ap_imw)], BBp_feat,
                                                   c.weights)
                        if d_coh <= d_app * (1 + (2 ** (level - c.max_levels)) * c.k):
                            p, i = p_coh, i_coh
                        else:
                            p, i = p_app, i_app
                Bp_pyr[level][row, col] = z['Ap_pyr'][int(i)][level][tuple(p)]
                s.append(p)
                im.append(int(i))
        out[level] = (np.array(s), np.array(im))
    return Bp_pyr, app_ix, coh


@pytest.mark.parametrize('name', ['g32', 'multiap'])
def test_minimal_integration_per_pixel_loop(name):
    from ia_amd import algorithms
    z = load_e2e(name)
    ch = 1 if z['A_pyr'][0].ndim == 2 else z['A_pyr'][0].shape[2]
    c = _cfg(ch, z['L'])
    c.weights, c.k = z['weights'], float(z['k'])
    flann, params, As, _ = algorithms.create_index(z['A_pyr'], z['Ap_pyr'], c)
    out = {}
    Bp, app_ix, coh = _reference_loop(z, c, flann, params, As, out)
    assert np.array_equal(np.array(app_ix), z['app_ix'])
    assert np.array_equal(np.array(coh), z['coh'])
    for level in range(1, z['L']):
        assert np.array_equal(out[level][0], z['s'][level]) and np.array_equal(out[level][1], z['im'][level])
        assert np.array_equal(Bp[level], z['Bp_final'][level])


def test_coherence_batch_matches_per_pixel_and_errors():
    """best_coherence_match_batch over a whole raster level (final s / im: every pixel's causal
    neighbours are final) equals the per-pixel calls; a short s raises (IndexError there)."""
    from ia_amd import _native, algorithms
    z = load_e2e('g64')
    L = z['L']
    level = L - 1
    c = _cfg(1, L)
    flann, params, As, _ = algorithms.create_index(z['A_pyr'], z['Ap_pyr'], c)
    B_features = algorithms.compute_feature_array(z['B_pyr'], c, full_feat=True)
    from ia_amd.img_preprocess import pad_img_pair
    h, w = z['B_pyr'][level].shape[:2]
    Bp_pd = pad_img_pair(z['Bp_final'][level - 1], z['Bp_final'][level], c)
    pxs = np.array([(r, col) for r in range(h) for col in range(w)])
    Q = np.array([np.hstack([B_features[level][r * w + col],
                             algorithms.extract_pixel_feature(Bp_pd, (r, col), c, full_feat=False)]) for r, col in pxs])
    s, im = z['s'][level], z['im'][level]
    A_hw = z['A_pyr'][level].shape[:2]
    p, img, rs = algorithms.best_coherence_match_batch(As[level], A_hw, Q, s, im, pxs, w, c)
    assert tuple(p[0]) == (-1, -1) and img[0] == 0 and tuple(rs[0]) == (0, 0)
    for qi in list(range(0, h * w, 37)) + [1, w, h * w - 1]:
        p1, i1, r1 = algorithms.best_coherence_match(As[level], A_hw, Q[qi], list(s[:qi]), list(im[:qi]), pxs[qi], w, c)
        assert (tuple(p1), i1, tuple(r1)) == (tuple(p[qi]), img[qi], tuple(rs[qi]))
    with pytest.raises(_native.IAError):
        algorithms.best_coherence_match_batch(As[level], A_hw, Q[w + 3:w + 4], s[:2], im[:2], pxs[w + 3:w + 4], w, c)


def test_coherence_per_pixel_matches_oracle():
    """best_coherence_match on a plain As array (no attached index: one upload per call) against
    the oracle's restatement of algorithms.py:92-130 on teacher-forced g32 states."""
    from ia_amd import algorithms as alg
    from oracle import ia_oracle as O
    z = load_e2e('g32')
    L = z['L']
    level = L - 1
    c = _cfg(1, L)
    As = O.build_db(z['A_pyr'], z['Ap_pyr'], level)
    Bf = O.feature_array(z['B_pyr'], level, True)
    h, w = z['B_pyr'][level].shape
    A_h, A_w = z['A_pyr'][level].shape
    s, im = z['s'][level], z['im'][level]
    for qi in range(1, h * w, 13):
        r, col = divmod(qi, w)
        Bp = O.state_at(z['Bp_final'][level], z['Bp_init'][level], qi)
        q = O.query_feature(Bf, z['Bp_final'][level - 1], Bp, r, col, w)
        got = alg.best_coherence_match(As, (A_h, A_w), q, [tuple(x) for x in s[:qi]], list(im[:qi]),
                                       np.array([r, col]), w, c)
        ref = O.coherence(As, A_h, A_w, q, s, im, r, col, w)
        assert tuple(np.asarray(got[0])) == tuple(ref[0]) and got[1] == ref[1]
