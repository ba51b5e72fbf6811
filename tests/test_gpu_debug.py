"""GPU parity of the debug=True records (image_analogies.py:141-153,224-253) against the
reference's own per-call outputs, captured by oracle/gen_golden.py while the real reference ran:
every best_approximate_match index ('app_ix'), every best_coherence_match return ('coh',
(-1, -1, 0) for "no candidate") and every compute_distance value ('dist', d_app then d_coh).

NN indices, coherence picks and distances must be bit-exact.  compute_distance =
norm((a - q) * w)**2: numpy's norm of a 1-D vector is sqrt(x.dot(x)), a BLAS ddot whose summation
order the kernels restate (blas_dot_sq in ia_kernels.hip; oracle blas_ddot_sq, pinned against
these vectors in tests/test_oracle_golden.py), and `** 2` on the numpy scalar is libm pow, which
the host applies to the kernel's dot (_native.Context.synthesize_level).
"""
import pickle

import numpy as np
import pytest

from golden_util import BIG_CASES, E2E_CASES, load_e2e

pytestmark = pytest.mark.gpu


def _run_debug(ctx, z, prune_all=False, variant=24):
    """prune_all: option prune_min_rows = 1, so every 1-channel level goes through the certified
    pruned scan (K2p -> K3p) instead of only DB levels of >= 2^19 rows; variant:
    the pruned-scan kernel (option k3p_variant; 24 = the library default)."""
    from ia_amd import _native
    L, k = z['L'], float(z['k'])
    Bp = [x.copy() for x in z['Bp_init']]
    out = {}
    st = _native.Stats()
    if prune_all:
        ctx.set_option('prune_min_rows', 1)
    ctx.set_option('k3p_variant', variant)
    try:
        for level in range(1, L):
            kf = 1 + (2 ** (level - L)) * k
            dbg = {}
            s, im = ctx.synthesize_level(z['A_pyr'][level], z['A_pyr'][level - 1], [p[level] for p in z['Ap_pyr']],
                                         [p[level - 1] for p in z['Ap_pyr']], z['B_pyr'][level],
                                         z['B_pyr'][level - 1], Bp[level - 1], Bp[level], z['weights'], kf, st,
                                         debug=dbg)
            out[level] = (s, im, dbg)
    finally:
        ctx.set_option('prune_min_rows', 524288)
        ctx.set_option('k3p_variant', 24)
    return out, Bp, st


@pytest.mark.parametrize('prune_all,variant', [(False, 24), (True, 20), (True, 21), (True, 22), (True, 24), (True, 25)],
                         ids=['default', 'pruned_v20', 'pruned_presorted_v21', 'pruned_v22', 'pruned_v24',
                              'pruned_presorted_v25'])
@pytest.mark.parametrize('name', E2E_CASES + BIG_CASES)
def test_debug_records_match_reference_calls(ctx, name, prune_all, variant):
    """Every NN pick, coherence pick and compute_distance value of the reference run.  With
    prune_all, the pruned scan K3p decides every 1-channel level (the bench's
    dominant kernel checked directly against the reference's own per-pixel picks).  Variants 21
    and 25 force the presorted wide-step path on every step: the per-step query sort K2s
    (k_query_sort) + the presorted scan - the kernels cfg4's 2048^2 level and every batched step
    wider than 512 queries run.  20 / 21: whole tiles; 22: the hi-only stream; 24 / 25: the
    two-pass scan (LDS-DMA hi stream, then the passing tiles' full chains)."""
    z = load_e2e(name)
    out, Bp, st = _run_debug(ctx, z, prune_all, variant)
    ch = 1 if z['A_pyr'][0].ndim == 2 else z['A_pyr'][0].shape[2]
    if prune_all:
        assert st.pruned_levels == (z['L'] - 1 if ch == 1 else 0)
    if st.pruned_levels > 0:  # the hi x hi block filter runs on pruned levels only
        assert 0 < st.dist_pairs_corrected <= st.dist_pairs
        assert 0 < st.dist_tiles_rows <= st.dist_tiles
    assert st.bound_violations == 0 and st.kappa_ambiguous == 0
    app, coh, dist = [], [], []
    for level in range(1, z['L']):
        s, im, dbg = out[level]
        assert np.array_equal(s, z['s'][level]) and np.array_equal(im, z['im'][level])
        assert np.array_equal(Bp[level], z['Bp_final'][level])
        src, d = dbg['src'], dbg['dist']
        a_h, a_w = z['A_pyr'][level].shape[:2]
        h, w = z['B_pyr'][level].shape[:2]
        app.extend((src[:, 2].astype(np.int64) * a_h + src[:, 0]) * a_w + src[:, 1])
        for qi in range(1, h * w):
            if src[qi, 5]:
                nb = src[qi, 3] * w + src[qi, 4]
                r, c = divmod(qi, w)
                coh.append((s[nb, 0] + r - src[qi, 3], s[nb, 1] + c - src[qi, 4], im[nb]))
                dist.extend(d[qi])
            else:
                assert src[qi, 3] == 0 and src[qi, 4] == 0 and d[qi, 0] == 0 and d[qi, 1] == 0
                coh.append((-1, -1, 0))
        assert src[0, 5] == 0   # the level's first pixel never consults coherence (:186-189)
    assert np.array_equal(np.array(app), z['app_ix'])
    assert np.array_equal(np.array(coh), z['coh'])
    dist = np.array(dist)
    assert dist.shape == z['dist'].shape
    print('%s: %d of %d compute_distance values bit-identical' % (name, int((dist == z['dist']).sum()), dist.size))
    assert np.array_equal(dist, z['dist'])


def test_main_debug_writes_reference_pickles(ctx, tmp_path):
    """image_analogies_main(debug=True) on the g32 golden inputs: the [sa, sc, rstars, s, im]
    pickles hold the reference's per-pixel lists (sa = every NN pick in raster order)."""
    from ia_amd import image_analogies as IA
    import types
    z = load_e2e('g32')
    c = types.SimpleNamespace(k=float(z['k']), weights=z['weights'], max_levels=z['L'])
    Bp = [x.copy() for x in z['Bp_init']]
    dbg = {}
    S, IM = IA.synthesize_pyramid(z['A_pyr'], z['Ap_pyr'], z['B_pyr'], Bp, c, ctx=ctx, debug=dbg)
    app = []
    for level in range(1, z['L']):
        h, w = Bp[level].shape[:2]
        d = IA.debug_structures(S[level], IM[level], dbg[level], (h, w))
        IA._save_debug(str(tmp_path) + '/', level, d, Bp[level], S[level], IM[level])
        with open(tmp_path / ('%d_srcs.pickle' % level), 'rb') as f:
            sa, sc, rstars, s_list, im_list = pickle.load(f)
        assert len(sa) == len(sc) == len(rstars) == len(s_list) == len(im_list) == h * w
        assert np.array_equal(np.array(s_list), z['s'][level]) and im_list == list(z['im'][level])
        a_w = z['A_pyr'][level].shape[1]
        app.extend(r * a_w + col for r, col in sa)           # one A' image: ix = r * a_w + c
        assert all((tmp_path / (p % level)).exists() for p in ['%d_psrc.eps', '%d_appdist.eps', '%d_cohdist.eps',
                                                                 '%d_output.eps', '%d_imgsrc.eps'])
        colours = {tuple(x) for x in d['p_src'].reshape(-1, 3)}
        assert colours <= {(1., 1., 0.), (1., 0., 0.), (0., 0., 0.)}
        assert tuple(d['p_src'][0, 0]) == (0., 0., 0.) and sc[0] == (0, 0) and rstars[0] == (0, 0)
    assert np.array_equal(np.array(app), z['app_ix'])
