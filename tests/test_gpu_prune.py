"""Certified pruned scan: the synthesis with pruning on must be bit-identical to
the unpruned exact scan on every level (source maps and B'), while contracting fewer
(DB tile, query tile) pairs.  The 512^2 job prunes its finest level, the 1024^2 job (cfg3, the
bench configuration) its two finest."""
import numpy as np
import pytest

import ia_amd  # noqa: F401

pytestmark = pytest.mark.gpu


def _run(ctx, job, prune, variant=22, group=1):
    from ia_amd import _native
    ctx.set_option('prune', prune)
    ctx.set_option('prune_group', group)
    ctx.set_option('k3p_variant', variant)
    ctx.set_option('prune_min_rows', 262144)  # prune the 512^2 level too (default: 1024^2 and up)
    Bp = [x.copy() for x in job.Bp_init]
    S, IM = {}, {}
    st = _native.Stats()
    try:
        for level in range(1, job.L):
            S[level], IM[level] = ctx.synthesize_level(
                job.A_pyr[level], job.A_pyr[level - 1], [p[level] for p in job.Ap_pyr_list],
                [p[level - 1] for p in job.Ap_pyr_list], job.B_pyr[level], job.B_pyr[level - 1], Bp[level - 1],
                Bp[level], job.weights, job.kappa_factor(level), st)
    finally:
        ctx.set_option('prune', 1)
        ctx.set_option('k3p_variant', 24)
        ctx.set_option('prune_min_rows', 524288)
        ctx.set_option('prune_group', 1)
    return Bp, S, IM, st


@pytest.mark.parametrize('size,n_pruned,variant', [(sz, n, v) for v in (20, 21, 22, 24, 25) for sz, n in ((512, 1), (1024, 2))])
def test_pruned_equals_unpruned(ctx, size, n_pruned, variant):
    """variant = the pruned-scan kernel version (option k3p_variant): 20 / 21 whole tiles, 22 the
    hi-only tile stream, 24 / 25 the two-pass scan (LDS-DMA hi stream, then the passing tiles'
    chains); the odd ones with the queries presorted once per step.  Every one is exact."""
    from ia_amd import synth
    job = synth.make_job(size)
    Bp0, S0, IM0, st0 = _run(ctx, job, 0)
    Bp1, S1, IM1, st1 = _run(ctx, job, 1, variant)
    assert st0.pruned_levels == 0 and st1.pruned_levels == n_pruned
    for level in range(1, job.L):
        assert np.array_equal(S0[level], S1[level]), level
        assert np.array_equal(IM0[level], IM1[level]), level
        assert np.array_equal(Bp0[level], Bp1[level]), level
    assert st1.bound_violations == 0 and st0.bound_violations == 0
    assert st1.dist_pairs < st1.dist_pairs_full
    assert st1.dist_pairs_full == st0.dist_pairs_full
    assert st1.dist_tiles <= st1.dist_tiles_full and st1.dist_tiles_full == st0.dist_tiles_full
    # every variant has the hi x hi block filter: most box-needed pairs stop after a cheap product
    assert 0 < st1.dist_pairs_corrected < st1.dist_pairs
    assert 0 < st1.dist_tiles_rows <= st1.dist_tiles   # loaded tiles with a filter-passing block
    print('filter-passing pairs %.3f of the box-needed ones, tiles %.3f of the loaded ones'
          % (st1.dist_pairs_corrected / st1.dist_pairs, st1.dist_tiles_rows / st1.dist_tiles))
    print('size %d: pairs left %.3f, DB tiles loaded %.3f, fallbacks %d -> %d'
          % (size, st1.dist_pairs / st1.dist_pairs_full, st1.dist_tiles / st1.dist_tiles_full, st0.fallbacks,
             st1.fallbacks))


@pytest.mark.parametrize('variant', [21, 22, 24, 25])
def test_fused_gather_equals_separate_launches(ctx, variant):
    """option fuse_gather (ia_kernels.hip k_merge_gather): the merge of step t and the gather of
    step t + 1 in one launch, the step's results handed row to row; with K3 timing every third
    step (time_dist 3: sampled steps run the separate launches) the fused and separate forms
    alternate within a level; option fuse_sort moves the query sort into the fused gathers.  All
    runs bit-identical (21 / 25: presorted wide-step scans)."""
    from ia_amd import synth
    job = synth.make_job(1024)
    runs = []
    # (fuse_gather, time_dist, fuse_sort): fuse_sort = the fused gathers also sort the next step
    # for the presorted scan (k_merge_gather sorted_publish), alone and mixed with sampled steps
    for fuse, stride, fsort in ((0, 0, 0), (1, 0, 0), (1, 3, 0), (1, 0, 1), (1, 3, 1)):
        ctx.set_option('fuse_gather', fuse)
        ctx.set_option('time_dist', stride)
        ctx.set_option('fuse_sort', fsort)
        try:
            runs.append(_run(ctx, job, 1, variant))
        finally:
            ctx.set_option('fuse_gather', 1)
            ctx.set_option('time_dist', 0)
            ctx.set_option('fuse_sort', 0)
    for Bp, S, IM, st in runs[1:]:
        for level in range(1, job.L):
            assert np.array_equal(S[level], runs[0][1][level]), level
            assert np.array_equal(IM[level], runs[0][2][level]), level
            assert np.array_equal(Bp[level], runs[0][0][level]), level
        assert st.bound_violations == 0 and st.pruned_levels == 2
        # rescans depend on which wave took which tile (dynamic hand-out): close, not equal
        assert abs(st.fallbacks - runs[0][3].fallbacks) <= 0.05 * runs[0][3].fallbacks + 10


@pytest.mark.parametrize('wgs', [128, 64])
def test_scan_workgroups_equal_default(ctx, wgs):
    """option scan_wgs (bench.py gives the coarser pipelined levels' contexts 128):
    the pruned and unpruned split-f16 scans on fewer workgroups (more DB tiles each, fewer records
    per query for the merge) give the same decisions on every level as one workgroup per CU"""
    from ia_amd import synth
    job = synth.make_job(512)
    Bp0, S0, IM0, st0 = _run(ctx, job, 1, 24)
    ctx.set_option('scan_wgs', wgs)
    try:
        Bp1, S1, IM1, st1 = _run(ctx, job, 1, 24)
    finally:
        ctx.set_option('scan_wgs', 256)
    for level in range(1, job.L):
        assert np.array_equal(S0[level], S1[level]), level
        assert np.array_equal(IM0[level], IM1[level]), level
        assert np.array_equal(Bp0[level], Bp1[level]), level
    assert st1.bound_violations == 0 and st1.pruned_levels == st0.pruned_levels == 1


def test_scan_workgroups_option_rejects_bad_values(ctx):
    from ia_amd import _native
    for bad in (0, 4, 12, 264):
        with pytest.raises(_native.IAError):
            ctx.set_option('scan_wgs', bad)


@pytest.mark.parametrize('size,group', [(512, 2), (1024, 4), (1024, 8)])
def test_pruned_groups_equal_unpruned(ctx, size, group):
    """option prune_group: Morton tiles interleaved in groups of G (sort neighbours in different
    tiles and workgroup chunks): a different DB layout, the same decisions on every level"""
    from ia_amd import synth
    job = synth.make_job(size)
    Bp0, S0, IM0, st0 = _run(ctx, job, 0)
    Bp1, S1, IM1, st1 = _run(ctx, job, 1, 24, group)
    for level in range(1, job.L):
        assert np.array_equal(S0[level], S1[level]), level
        assert np.array_equal(IM0[level], IM1[level]), level
        assert np.array_equal(Bp0[level], Bp1[level]), level
    assert st1.bound_violations == 0 and st1.pruned_levels >= 1
    print('group %d: pairs left %.3f, DB tiles loaded %.3f, fallbacks %d' % (
        group, st1.dist_pairs / st1.dist_pairs_full, st1.dist_tiles / st1.dist_tiles_full, st1.fallbacks))


def test_prune_option_rejects_bad_values(ctx):
    from ia_amd import _native
    with pytest.raises(_native.IAError):
        ctx.set_option('prune', 2)
    with pytest.raises(_native.IAError):
        ctx.set_option('prune_group', 3)
    for v in (1, 6, 7, 11, 12, 13, 14, 15, 16, 17, 18, 19, 23, 26):   # earlier versions: in git history only
        with pytest.raises(_native.IAError):
            ctx.set_option('k3p_variant', v)
    with pytest.raises(_native.IAError):
        ctx.set_option('prune_min_rows', 0)


@pytest.mark.parametrize('variant', [20, 21, 22, 24, 25])
def test_pruned_scan_over_512_tiles_per_workgroup(ctx, variant):
    """a DB of more than 256 x 512 tiles (> 4.19 M rows: here A 2048 x 2080,
    133,120 tiles, 520 per workgroup) against a small B.  The pruned scan keeps every workgroup's
    tile boxes in LDS (up to IA_K3P_MAXK_LDS tiles); every tile must be scanned, in the
    in-kernel-sort (20, 22, 24) and the presorted (21, 25) forms (24 / 25: beyond the LDS budget of
    their static DMA rings the launcher takes 22 / 21): the level must equal the unpruned scan bit
    for bit."""
    from ia_amd import _native, synth
    from ia_amd import config as _c
    ah, aw, bh, bw = 2048, 2080, 48, 48
    A = synth.smooth(ah, aw, 2, 1)
    Ap = synth.filt(A)
    Ac, Apc = np.ascontiguousarray(A[::2, ::2]), np.ascontiguousarray(Ap[::2, ::2])
    B = synth.smooth(bh, bw, 2, 2)
    Bc = np.ascontiguousarray(B[::2, ::2])
    rs = np.random.RandomState(7)
    Bpc, Bp_init = rs.rand(bh // 2, bw // 2), rs.rand(bh, bw)
    w = _c.compute_weights(_c.n_sm, _c.n_lg, _c.n_half, 1)
    assert -(-ah * aw // 32) > 256 * 512
    out = []
    for prune in (0, 1):
        Bp = Bp_init.copy()
        st = _native.Stats()
        ctx.set_option('prune', prune)
        ctx.set_option('prune_min_rows', 1)
        ctx.set_option('k3p_variant', variant)
        try:
            s, im = ctx.synthesize_level(A, Ac, [Ap], [Apc], B, Bc, Bpc, Bp, w, 1.25, st)
        finally:
            ctx.set_option('prune', 1)
            ctx.set_option('prune_min_rows', 524288)
            ctx.set_option('k3p_variant', 24)
        out.append((s, im, Bp, st))
    (s0, im0, Bp0, st0), (s1, im1, Bp1, st1) = out
    assert st0.pruned_levels == 0 and st1.pruned_levels == 1
    assert st1.bound_violations == 0 and st0.bound_violations == 0
    assert np.array_equal(s0, s1) and np.array_equal(im0, im1) and np.array_equal(Bp0, Bp1)
    assert st1.dist_tiles < st1.dist_tiles_full


@pytest.mark.parametrize('opt', ['fuse_sort'])
@pytest.mark.parametrize('name', ['g64', 'ties128', 'k25', 'g256'])
def test_fused_sort_matches_reference(ctx, name, opt):
    """option fuse_sort with every level pruned: each fused merge + gather ranks the next step's
    keys across its waves and writes the presorted scan inputs (ia_kernels.hip sorted_publish);
    s, im and B' of every level equal the reference run's."""
    from ia_amd import _native
    from golden_util import BIG_CASES, E2E_CASES, load_e2e
    if name not in E2E_CASES + BIG_CASES:
        pytest.skip('fixture absent')
    z = load_e2e(name)
    L, k = z['L'], float(z['k'])
    Bp = [x.copy() for x in z['Bp_init']]
    st = _native.Stats()
    ctx.set_option('prune_min_rows', 1)
    ctx.set_option(opt, 1)
    try:
        for level in range(1, L):
            s, im = ctx.synthesize_level(z['A_pyr'][level], z['A_pyr'][level - 1], [p[level] for p in z['Ap_pyr']],
                                         [p[level - 1] for p in z['Ap_pyr']], z['B_pyr'][level], z['B_pyr'][level - 1],
                                         Bp[level - 1], Bp[level], z['weights'], 1 + 2.0 ** (level - L) * k, st)
            assert np.array_equal(s, z['s'][level]) and np.array_equal(im, z['im'][level]), level
            assert np.array_equal(Bp[level], z['Bp_final'][level]), level
    finally:
        ctx.set_option('prune_min_rows', 524288)
        ctx.set_option(opt, 0)
    assert st.bound_violations == 0 and st.kappa_ambiguous == 0 and st.pruned_levels == L - 1


def test_nn_bound_is_exact_and_tighter(ctx):
    """option nn_bound (default on): the gathers also bound U' by the causal neighbours' exact NN
    rows, shifted.  Exact with and without it (the 1024^2 job's two pruned levels: s, im and B'
    identical), and the scan contracts fewer pairs with it (a smaller radius per query)."""
    from ia_amd import synth
    job = synth.make_job(1024)
    ctx.set_option('nn_bound', 0)
    try:
        Bp0, S0, IM0, st0 = _run(ctx, job, 1, 24)
    finally:
        ctx.set_option('nn_bound', 1)
    Bp1, S1, IM1, st1 = _run(ctx, job, 1, 24)
    for level in range(1, job.L):
        assert np.array_equal(S0[level], S1[level]), level
        assert np.array_equal(IM0[level], IM1[level]), level
        assert np.array_equal(Bp0[level], Bp1[level]), level
    assert st0.bound_violations == 0 and st1.bound_violations == 0
    assert st1.dist_pairs < st0.dist_pairs
    print('pairs %.4f -> %.4f of the full scan, corrected %.4f -> %.4f, fallbacks %d -> %d'
          % (st0.dist_pairs / st0.dist_pairs_full, st1.dist_pairs / st1.dist_pairs_full,
             st0.dist_pairs_corrected / st0.dist_pairs_full, st1.dist_pairs_corrected / st1.dist_pairs_full,
             st0.fallbacks, st1.fallbacks))

