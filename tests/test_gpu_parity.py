"""GPU parity: the HIP path (through the C ABI) against the reference's own outputs.

Golden end-to-end fixtures (tests/golden/e2e_*.npz) were produced by running the real reference
(oracle/gen_golden.py): the round-1 cases up to 64x64 and the round-2 cases cfg1 (BASELINE
config 1's 117x180 YIQ stand-in), g128, g256, ties128 and k25 (kappa 25).  Fed the same pyramids, B' initialisation and weights, the GPU level
path must reproduce every level's source map s, image map im and final B' BIT-EXACTLY: the NN
is exact (certified MFMA + fp64 rerank in numpy's summation order), coherence distances are
bit-identical, and the kappa test's weighted distances follow the golden host's BLAS dot order
(tests/test_gpu_debug.py checks every one of them bit-exactly).
"""
import numpy as np
import pytest

from golden_util import BIG_CASES, E2E_CASES, SLIM_CASES, load_e2e

pytestmark = pytest.mark.gpu


@pytest.fixture(params=['f16x3', 'f32'])
def matcher(request, ctx):
    """Every certified matcher (split-f16 MFMA with the packed-index K3 epilogue, fp32 MFMA)
    must give the reference's decisions."""
    from ia_amd import _native
    ctx.set_option('matcher', _native.IA_MATCH_F32 if request.param == 'f32' else _native.IA_MATCH_F16X3)
    yield request.param
    ctx.set_option('matcher', _native.IA_MATCH_F16X3)


def _run_levels(ctx, z, Bp, A_pyr=None, Ap_pyr=None, B_pyr=None):
    from ia_amd import _native
    A_pyr, Ap_pyr, B_pyr = A_pyr or z['A_pyr'], Ap_pyr or z['Ap_pyr'], B_pyr or z['B_pyr']
    L, k = z['L'], float(z['k'])
    st = _native.Stats()
    out = {}
    for level in range(1, L):
        kf = 1 + (2 ** (level - L)) * k
        out[level] = ctx.synthesize_level(A_pyr[level], A_pyr[level - 1], [p[level] for p in Ap_pyr],
                                          [p[level - 1] for p in Ap_pyr], B_pyr[level], B_pyr[level - 1],
                                          Bp[level - 1], Bp[level], z['weights'], kf, st)
    return out, st


@pytest.fixture(params=[0], ids=['rowdb'])
def row_source(request, ctx):
    """exact rows of the rerank / coherence / bound from the fp64 row DB (the A-image gather of
    round 2, measured slower, is in git history)"""
    ctx.set_option('row_source', request.param)
    yield request.param


@pytest.mark.parametrize('name', E2E_CASES + BIG_CASES)
def test_level_path_matches_reference(ctx, matcher, row_source, name):
    z = load_e2e(name)
    Bp = [x.copy() for x in z['Bp_init']]
    out, st = _run_levels(ctx, z, Bp)
    for level, (s, im) in out.items():
        assert np.array_equal(s, z['s'][level]), 'level %d source map differs' % level
        assert np.array_equal(im, z['im'][level]), 'level %d image map differs' % level
        assert np.array_equal(Bp[level], z['Bp_final'][level]), 'level %d B\' differs' % level
    assert st.bound_violations == 0
    assert st.kappa_ambiguous == 0
    ch = 1 if z['A_pyr'][0].ndim == 2 else z['A_pyr'][0].shape[2]
    assert st.f16_levels == (z['L'] - 1 if (matcher == 'f16x3' and ch < 3) else 0)


def test_split_f16_falls_back_to_fp32_outside_f16_range(ctx):
    """Image values beyond +-64 would overflow the split-f16 operands: the level runs on the
    fp32 matcher instead, with the same (oracle) decisions."""
    from oracle import ia_oracle as O
    z = load_e2e('g24k5')
    sc = lambda pyr: [x * 100.0 for x in pyr]
    A_pyr, Ap_pyr, B_pyr = sc(z['A_pyr']), [sc(p) for p in z['Ap_pyr']], sc(z['B_pyr'])
    Bp0 = sc(z['Bp_init'])
    Bp_gpu, Bp_cpu = [x.copy() for x in Bp0], [x.copy() for x in Bp0]
    out, st = _run_levels(ctx, z, Bp_gpu, A_pyr, Ap_pyr, B_pyr)
    S, IM = O.run_all_levels(A_pyr, Ap_pyr, B_pyr, Bp_cpu, float(z['k']), z['weights'])
    assert st.f16_levels == 0
    for level, (s, im) in out.items():
        assert np.array_equal(s, S[level]) and np.array_equal(im, IM[level])
        assert np.array_equal(Bp_gpu[level], Bp_cpu[level])


def _numpy_nn(pts, q):
    d = ((pts[None, :, :] - q[:, None, :]) ** 2).sum(axis=2)
    return d.argmin(axis=1), d.min(axis=1)


@pytest.mark.parametrize('n,d,nq,seed', [(1, 55, 5, 0), (33, 55, 40, 1), (5000, 55, 300, 2), (4099, 21, 70, 3),
                                         (2000, 165, 50, 4), (700, 110, 33, 5)])
def test_exact_index_matches_numpy(ctx, n, d, nq, seed):
    from ia_amd import _native
    rs = np.random.RandomState(seed)
    pts = rs.rand(n, d)
    q = rs.rand(nq, d)
    q[: min(nq, n) // 2] = pts[: min(nq, n) // 2]  # exact hits (distance 0)
    idx = _native.ExactIndex(ctx, pts)
    i_gpu, d_gpu = idx.query(q)
    for j in range(nq):
        dd = ((pts - q[j]) ** 2).sum(axis=1)
        assert i_gpu[j] == int(np.argmin(dd))
        assert d_gpu[j] == dd[i_gpu[j]]


def test_exact_index_ties_lowest_index(ctx):
    from ia_amd import _native
    rs = np.random.RandomState(7)
    base = rs.rand(50, 55)
    pts = np.vstack([base] * 40)  # every row duplicated 40 times -> exact ties
    rs.shuffle(pts)
    q = base + 1e-3 * rs.rand(*base.shape)
    i_gpu, _ = _native.ExactIndex(ctx, pts).query(q)
    for j in range(len(q)):
        dd = ((pts - q[j]) ** 2).sum(axis=1)
        assert i_gpu[j] == int(np.argmin(dd))


@pytest.mark.parametrize('name', SLIM_CASES)
def test_slim_reference_runs_with_product_defaults(ctx, name):
    """Reference runs in 'slim' fixtures (oracle/gen_golden.py run_case slim=True): g512 is
    BASELINE config 2's shape (512^2, the finest 5 pyramid levels), where the product's default
    path runs the certified pruned scan on the 512^2 level (262,144 DB rows >= the bench's
    prune_min_rows) -
    the bench's dominant kernel pinned end to end to the reference; g64slim
    checks the slim writer and the level cap on a 4-level 64^2 run.  Every level's s and im must
    equal the reference's exactly, and every B' level its sha1."""
    from golden_util import load_slim, sha1_f64
    z = load_slim(name)
    Bp = [x.copy() for x in z['Bp_init']]
    # the bench's setting for every configuration whose 512^2 levels it runs (cfg3 pipelined, cfg4,
    # cfg5: bench.py --prune-min-rows 262144), so the 512^2 level runs the pruned scan K3p
    ctx.set_option('prune_min_rows', 262144)
    try:
        out, st = _run_levels(ctx, z, Bp)
    finally:
        ctx.set_option('prune_min_rows', 524288)
    for level, (s, im) in out.items():
        assert np.array_equal(s, z['s'][level]), 'level %d source map differs' % level
        assert np.array_equal(im, z['im'][level]), 'level %d image map differs' % level
        assert sha1_f64(Bp[level]) == z['sha1']['Bp_%d' % level], 'level %d B\' differs' % level
    assert st.bound_violations == 0 and st.kappa_ambiguous == 0
    if name == 'g512':
        assert st.pruned_levels >= 1, 'the 512^2 level must run the pruned scan under the product defaults'
