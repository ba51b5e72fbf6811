"""The oracle (oracle/ia_oracle.py, CPU restatement) is pinned against the reference's own
outputs: golden vectors produced by running the real reference (oracle/gen_golden.py)."""
import os

import numpy as np
import pytest

from golden_util import E2E_CASES, GOLDEN, load_e2e
from oracle import ia_oracle as O


@pytest.mark.parametrize('name', [c for c in E2E_CASES if c != 'g64'] + [pytest.param('g64', marks=pytest.mark.slow)])
def test_oracle_reproduces_reference_end_to_end(name):
    z = load_e2e(name)
    w = z['weights']
    assert np.allclose(O.compute_weights(O.nch(z['A_pyr'][0])), w, rtol=1e-14, atol=0)
    Bp = [x.copy() for x in z['Bp_init']]
    log = []
    S, IM = O.run_all_levels(z['A_pyr'], z['Ap_pyr'], z['B_pyr'], Bp, float(z['k']), w, log=log)
    assert np.array_equal(np.array([x[0] for x in log]), z['app_ix'])           # every NN index
    coh = np.array([(x[1][0][0], x[1][0][1], x[1][1]) for x in log if x[1]])
    assert np.array_equal(np.array([v for x in log if x[1] for v in x[1][2:]]), z['dist'])  # weighted d
    for level in range(1, z['L']):
        assert np.array_equal(S[level], z['s'][level])
        assert np.array_equal(IM[level], z['im'][level])
        assert np.array_equal(Bp[level], z['Bp_final'][level])
    assert len(coh) <= len(z['coh'])


def test_oracle_feature_layout_kats():
    """algorithms_test.py:10-115 inputs (4x5 / 7x10, 1 and 3 channels) + random 3-level DBs."""
    g = np.load(os.path.join(GOLDEN, 'features.npz'))
    for ch in (1, 3):
        shp = (lambda h, w: (h, w) if ch == 1 else (h, w, ch))
        sm = 0.5 * np.ones(shp(4, 5)); sm[0, 0] = 0
        lg = 0.3 * np.ones(shp(7, 10)); lg[0, 0] = 1
        assert np.array_equal(O.feature_array([sm, lg], 1, True), g['c%d_full' % ch])
        assert np.array_equal(O.feature_array([sm, lg], 1, False), g['c%d_half' % ch])
        tag = 'rand_c%d' % ch
        A = [g['%s_A_%d' % (tag, l)] for l in range(3)]
        Ap = [g['%s_Ap_%d' % (tag, l)] for l in range(3)]
        for l in (1, 2):
            assert np.array_equal(O.build_db(A, [Ap], l), g['%s_As_%d' % (tag, l)])
        As = g['%s_As_2' % tag]
        Bf = O.feature_array(A, 2, True)
        h, w = A[2].shape[:2]
        Q = np.array([O.query_feature(Bf, Ap[1], Ap[2], r, c, w) for r in range(h) for c in range(w)])
        assert np.array_equal(Q, g['%s_Q_2' % tag])
        assert np.array_equal([O.nn_exact(As, q)[0] for q in Q], g['%s_nn_2' % tag])


def test_decide_pixel_teacher_forcing_matches_reference():
    """decide_pixel (the teacher-forcing checker used on GPU state) re-derives the reference's
    decisions from the final state of a golden run."""
    z = load_e2e('g32')
    L, k, w = z['L'], float(z['k']), z['weights']
    level = L - 1
    As = O.build_db(z['A_pyr'], z['Ap_pyr'], level)
    Bf = O.feature_array(z['B_pyr'], level, True)
    A_h, A_w = z['A_pyr'][level].shape[:2]
    h, wd = z['B_pyr'][level].shape[:2]
    s, im = z['s'][level], z['im'][level]
    for qi in range(0, h * wd, 7):
        r, c = divmod(qi, wd)
        out = O.decide_pixel(As, Bf, z['Bp_final'][level - 1], z['Bp_final'][level], z['Bp_init'][level], s, im,
                             A_h, A_w, level, L, k, w, r, c)
        (pr, pc), img = out['choice']
        assert (pr, pc, img) == (s[qi, 0], s[qi, 1], im[qi])


def test_blas_dot_order_reproduces_reference_distances(monkeypatch):
    """Every compute_distance value the reference produced (golden 'dist') is reproduced
    bit-for-bit by the explicit BLAS ddot order the GPU kernels restate (blas_ddot_sq), so the
    kappa rule's inputs, not only its decisions, are pinned independently of the host's BLAS."""
    z = load_e2e('g24k5')
    monkeypatch.setattr(O, 'compute_distance', O.compute_distance_blas)
    Bp = [x.copy() for x in z['Bp_init']]
    log = []
    O.run_all_levels(z['A_pyr'], z['Ap_pyr'], z['B_pyr'], Bp, float(z['k']), z['weights'], log=log)
    assert np.array_equal(np.array([v for x in log if x[1] for v in x[1][2:]]), z['dist'])


def test_blas_dot_order_three_channel():
    """D = 165 (3 channels) and 110: the same restatement against the host's np.dot on the rgb3
    golden weights (skipped where numpy's BLAS uses another kernel)."""
    rng = np.random.default_rng(5)
    x = rng.standard_normal((40, 165)) * rng.uniform(0, 1, (40, 165))
    got = [O.blas_ddot_sq(v) for v in x]
    ref = [float(v.dot(v)) for v in x]
    if got != ref:
        pytest.skip('this host numpy BLAS sums in another order (not the golden-generating kernel)')
    assert got == ref


def test_libm_pow_square_differs_from_product_only_near_midpoints():
    """compute_distance ends in `norm(...) ** 2` on a numpy scalar = libm pow(y, 2.0), which is
    not always the correctly rounded y * y the kernels use.  K4's audit (pow2_alt in
    ia_kernels.hip, ia_stats.kappa_ambiguous) assumes every difference lies where the exact
    square is within 0.9 half-ulp of a rounding midpoint and equals the neighbour toward it:
    checked here against this host's libm on random y."""
    import math
    from fractions import Fraction
    rng = np.random.default_rng(11)
    ys = rng.uniform(0, 1, 100000) * 10.0 ** rng.integers(-6, 3, 100000)
    n_diff = 0
    for y in ys.tolist():
        p, h = y ** 2, y * y
        lo = float(Fraction(y) * Fraction(y) - Fraction(h))
        half = math.ulp(h) / 2
        alt = h if abs(lo) < 0.9 * half else math.nextafter(h, math.inf if lo > 0 else 0.0)
        assert p in (h, alt)
        n_diff += p != h
    assert n_diff > 0   # the effect is real (about 1 in 1000) ...
    assert n_diff < 1000


def test_oracle_reproduces_slim_reference_run():
    """The slim fixture format (oracle/gen_golden.py run_case slim=True, the g512 case's format)
    on its 64^2 / 4-level check case: the reference's pyramids, the product's seeded B' init
    (hash-checked by load_slim), and the oracle's s / im / B' equal to the reference's."""
    from golden_util import load_slim, sha1_f64
    from oracle import ia_oracle as O
    z = load_slim('g64slim')
    Bp = [x.copy() for x in z['Bp_init']]
    S, IM = O.run_all_levels(z['A_pyr'], z['Ap_pyr'], z['B_pyr'], Bp, z['k'], z['weights'])
    for level in range(1, z['L']):
        assert np.array_equal(S[level], z['s'][level])
        assert np.array_equal(IM[level], z['im'][level])
        assert sha1_f64(Bp[level]) == z['sha1']['Bp_%d' % level]
