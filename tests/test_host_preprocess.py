"""Host-side (★H) preprocessing of the product package against the reference's outputs:
weights, pyramids (skimage 0.18.3 semantics restated), YIQ, remap, seeded B' init, codec,
and the reference-API array helpers of algorithms.py."""
import os

import numpy as np
import pytest

import ia_amd  # noqa: F401
from ia_amd import algorithms as alg
from ia_amd import config as c
from ia_amd import img_preprocess as ip
from golden_util import GOLDEN, load_e2e
from oracle import ia_oracle as O


def test_weights_match_reference():
    g = np.load(os.path.join(GOLDEN, 'weights.npz'))
    # exp() of numpy 1.26 (reference run) and 2.x may differ in the last ulp
    assert np.allclose(c.compute_weights(3, 5, 12, 1), g['w1'], rtol=1e-14, atol=0)
    assert np.allclose(c.compute_weights(3, 5, 12, 3), g['w3'], rtol=1e-14, atol=0)
    # config_test.py:21-30 sums
    w = c.compute_weights(3, 5, 12, 1)
    assert np.isclose(w[:9].sum(), 1. / 9) and np.isclose(w[9:34].sum(), 1. / 25)
    assert w[43:].sum() < 0.5 / 12


def test_pyramids_match_skimage_0_18():
    """Tolerance 1e-12: skimage estimates its resize transform by least squares (last-ulp
    differences in the bilinear coordinates); shapes and level counts must match exactly."""
    g = np.load(os.path.join(GOLDEN, 'pyramids.npz'))
    i = 0
    while 'img_%d' % i in g:
        pyr = ip.compute_gaussian_pyramid(g['img_%d' % i], 3)
        assert len(pyr) == int(g['n_%d' % i])
        for l, p in enumerate(pyr):
            ref = g['pyr_%d_%d' % (i, l)]
            assert p.shape == ref.shape
            assert np.abs(p - ref).max() < 1e-12
        i += 1


def test_pyramid_n_levels_cap():
    img = np.random.RandomState(0).rand(64, 64)
    assert len(ip.compute_gaussian_pyramid(img, 3)) == 6
    pyr = ip.compute_gaussian_pyramid(img, 3, n_levels=3)
    assert [p.shape for p in pyr] == [(16, 16), (32, 32), (64, 64)]


def test_color_and_remap_match_reference():
    g = np.load(os.path.join(GOLDEN, 'color.npz'))
    assert np.array_equal(ip.convert_to_YIQ(g['rgb']), g['yiq'])
    assert np.array_equal(ip.convert_to_RGB(ip.convert_to_YIQ(g['rgb'])), g['back'])
    assert np.allclose(ip.convert_to_RGB(ip.convert_to_YIQ(g['rgb'])), g['rgb'], atol=0.05)  # img_preprocess_test.py:9
    A, Ap = ip.remap_luminance(g['A'], [g['Ap']], g['B'])
    assert np.array_equal(A, g['A_remap']) and np.array_equal(Ap[0], g['Ap_remap'])
    with pytest.raises(ValueError):
        ip.convert_to_YIQ(g['rgb'] * 2)


def test_initialize_Bp_seeded_matches_reference_draw_order():
    z = load_e2e('g32')   # the golden run called np.random.seed(seed) then initialize_Bp
    Bp = ip.initialize_Bp(z['B_pyr'], init_rand=True, seed=int(z['seed']))
    for a, b in zip(Bp, z['Bp_init']):
        assert np.array_equal(a, b)
    copy = ip.initialize_Bp(z['B_pyr'], init_rand=False)
    for a, b in zip(copy, z['B_pyr']):
        assert np.array_equal(a, b) and a is not b


def test_index_codec_round_trip():
    h, w = 7, 11
    ix = np.arange(3 * h * w)
    (r, col), img = ip.Ap_ix2px(ix, h, w)
    assert np.array_equal(ip.Ap_px2ix((r, col), img, h, w), ix)
    assert np.array_equal(ip.px2ix(ip.ix2px(ix[:h * w], w), w), ix[:h * w])


def _setup(img):
    c.num_ch, c.padding_sm, c.padding_lg, c.weights = c.setup_vars(img)


def test_feature_array_and_pixel_feature_kats():
    """algorithms_test.py:10-115 restated against the golden outputs."""
    g = np.load(os.path.join(GOLDEN, 'features.npz'))
    for ch in (1, 3):
        shp = (lambda h, w: (h, w) if ch == 1 else (h, w, ch))
        sm = 0.5 * np.ones(shp(4, 5)); sm[0, 0] = 0
        lg = 0.3 * np.ones(shp(7, 10)); lg[0, 0] = 1
        _setup(lg)
        full = alg.compute_feature_array([sm, lg], c, full_feat=True)
        half = alg.compute_feature_array([sm, lg], c, full_feat=False)
        assert full[0] == [] and np.array_equal(full[1], g['c%d_full' % ch])
        assert np.array_equal(half[1], g['c%d_half' % ch])
        pd = ip.pad_img_pair(sm, lg, c)
        assert np.array_equal(alg.extract_pixel_feature(pd, (0, 0), c, True), g['c%d_px00_full' % ch])
        assert np.array_equal(alg.extract_pixel_feature(pd, (0, 0), c, False), g['c%d_px00_half' % ch])


def test_distance_helper_matches_oracle():
    """compute_distance (host numpy); best_coherence_match runs on the GPU (ia_coherence_batch),
    its oracle check is tests/test_gpu_flann_api.py::test_coherence_per_pixel_matches_oracle."""
    z = load_e2e('g32')
    L = z['L']
    level = L - 1
    _setup(z['A_pyr'][0])
    As = O.build_db(z['A_pyr'], z['Ap_pyr'], level)
    Bf = O.feature_array(z['B_pyr'], level, True)
    h, w = z['B_pyr'][level].shape
    A_h, A_w = z['A_pyr'][level].shape
    s, im = z['s'][level], z['im'][level]
    for qi in range(1, h * w, 13):
        r, col = divmod(qi, w)
        Bp = O.state_at(z['Bp_final'][level], z['Bp_init'][level], qi)
        q = O.query_feature(Bf, z['Bp_final'][level - 1], Bp, r, col, w)
        assert alg.compute_distance(As[5], q, z['weights']) == O.compute_distance(As[5], q, z['weights'])


def test_debug_structures_from_records():
    """debug=True bookkeeping (image_analogies.py:224-246) from per-pixel GPU records on a 2x3
    level: sc = s[r_star] + q - r_star where a coherence candidate existed, (0, 0) otherwise;
    p_src colours by which candidate won; img_src = im / max(im) (nan for one A' image)."""
    from ia_amd.image_analogies import debug_structures
    S = np.array([[4, 4], [4, 5], [7, 7], [5, 4], [5, 6], [1, 1]], dtype=np.int32)
    IM = np.zeros(6, dtype=np.int32)
    src = np.zeros((6, 6), dtype=np.int32)
    src[:, 0], src[:, 1] = S[:, 0], S[:, 1]
    src[2, :2] = (7, 7)
    src[1, 3:] = (0, 0, 1)        # r_star (0,0): p_coh = (4,4) + (0,1) = (4,5) = s[1] -> coherence won
    src[2, 3:] = (0, 1, 1)        # p_coh = (4,5) + (0,1) = (4,6) != s[2] -> NN won
    src[4, 3:] = (1, 0, 1)        # p_coh = (5,4) + (0,1) = (5,5) != s[4] = (5,6) -> NN
    src[4, :2] = (5, 6)
    dist = np.zeros((6, 2))
    dist[1], dist[2], dist[4] = (2., 1.), (1., 3.), (0.5, 0.75)
    d = debug_structures(S, IM, {'src': src, 'dist': dist}, (2, 3))
    assert d['sc'] == [(0, 0), (4, 5), (4, 6), (0, 0), (5, 5), (0, 0)]
    assert d['rstars'] == [(0, 0), (0, 0), (0, 1), (0, 0), (1, 0), (0, 0)]
    assert d['sa'][2] == (7, 7)
    assert [tuple(x) for x in d['p_src'].reshape(-1, 3)] == [(0, 0, 0), (1, 1, 0), (1, 0, 0), (0, 0, 0), (1, 0, 0),
                                                            (0, 0, 0)]
    assert d['app_dist'][0, 1] == 2. and d['coh_dist'][1, 1] == 0.75 and d['app_dist'][1, 0] == 0.
    assert np.isnan(d['img_src']).all()
