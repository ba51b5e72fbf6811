"""The sharded device path on one GPU (option "shard_emulate" = W): the A DB
of every level with >= 64 W tiles is split into W shards; each shard's distance scan and
certified per-shard winner (k_merge_level<FUSED=false>) run in turn, then the multi-rank finish
(k_finish_level: global winner = smallest exact distance, lowest row; coherence, kappa,
writeback) - everything the RCCL path runs except the all-gather itself.  Pruned levels keep
pruning under sharding (shard r = Morton tiles r, r + W, ..., stored contiguously).  Results must
be bit-identical to the reference (golden runs) and to unsharded runs (1024^2).
exchange = 1: the one-shot peer-write exchange instead (k_merge_xchg: each shard's winner is
written into the exchange slots with a release store, the last shard's launch polls the W slots
of every query with acquire loads and finishes the pixel) - the multi-rank kernels with the
peers' buffers aliased to this process's own."""
import numpy as np
import pytest

from golden_util import BIG_CASES, load_e2e

pytestmark = pytest.mark.gpu


def _run(ctx, z, W, prune_all, exchange=0, shard_unpruned=1):
    from ia_amd import _native
    L, k = z['L'], float(z['k'])
    Bp = [x.copy() for x in z['Bp_init']]
    st = _native.Stats()
    out = {}
    ctx.set_option('shard_emulate', W)
    ctx.set_option('exchange', exchange)
    ctx.set_option('shard_unpruned', shard_unpruned)
    if prune_all:
        ctx.set_option('prune_min_rows', 1)
    try:
        for level in range(1, L):
            out[level] = ctx.synthesize_level(z['A_pyr'][level], z['A_pyr'][level - 1], [p[level] for p in z['Ap_pyr']],
                                              [p[level - 1] for p in z['Ap_pyr']], z['B_pyr'][level],
                                              z['B_pyr'][level - 1], Bp[level - 1], Bp[level], z['weights'],
                                              1 + 2.0 ** (level - L) * k, st)
    finally:
        ctx.set_option('shard_emulate', 1)
        ctx.set_option('exchange', 0)
        ctx.set_option('shard_unpruned', 0)
        ctx.set_option('prune_min_rows', 524288)
    return out, Bp, st


@pytest.mark.parametrize('exchange', [0, 1], ids=['allgather', 'peerwrite'])
@pytest.mark.parametrize('prune_all', [False, True], ids=['unpruned', 'pruned'])
@pytest.mark.parametrize('W', [2, 4, 8])
@pytest.mark.parametrize('name', ['g64', 'ties128'] + [c for c in ('g128', 'g256') if c in BIG_CASES])
def test_emulated_shards_match_reference(ctx, name, W, prune_all, exchange):
    z = load_e2e(name)
    out, Bp, st = _run(ctx, z, W, prune_all, exchange)
    for level, (s, im) in out.items():
        assert np.array_equal(s, z['s'][level]) and np.array_equal(im, z['im'][level]), level
        assert np.array_equal(Bp[level], z['Bp_final'][level]), level
    assert st.bound_violations == 0 and st.kappa_ambiguous == 0


@pytest.mark.parametrize('W,exchange', [(4, 0), (8, 0), (2, 1), (8, 1)])
def test_emulated_shards_1024_match_unsharded(ctx, W, exchange):
    """cfg3 (pruned 1024^2 level, unpruned 512^2 level): W-way sharded == unsharded, every level."""
    from ia_amd import synth
    job = synth.make_job(1024)
    z = {'L': job.L, 'k': job.k, 'A_pyr': job.A_pyr, 'Ap_pyr': job.Ap_pyr_list, 'B_pyr': job.B_pyr,
         'Bp_init': job.Bp_init, 'weights': job.weights}
    ref, Bp_ref, _ = _run(ctx, z, 1, False)
    out, Bp, st = _run(ctx, z, W, False, exchange)
    for level in range(1, job.L):
        assert np.array_equal(out[level][0], ref[level][0]) and np.array_equal(out[level][1], ref[level][1]), level
        assert np.array_equal(Bp[level], Bp_ref[level]), level
    assert st.pruned_levels == 1 and st.bound_violations == 0


def test_shard_emulate_option_bounds(ctx):
    from ia_amd import _native
    for bad in (0, 65):
        with pytest.raises(_native.IAError):
            ctx.set_option('shard_emulate', bad)


def test_exchange_option_bounds(ctx):
    from ia_amd import _native
    with pytest.raises(_native.IAError):
        ctx.set_option('exchange', 3)
    ctx.set_option('exchange', 1)
    ctx.set_option('shard_emulate', 32)   # more shards than exchange slots: refused per level
    ctx.set_option('prune_min_rows', 1)   # a pruned level shards (shard_unpruned = 0)
    try:
        z = load_e2e('g256')   # 2048 tiles at 256^2: a 32-way emulated shard level
        with pytest.raises(_native.IAError):
            L = z['L']
            ctx.synthesize_level(z['A_pyr'][L - 1], z['A_pyr'][L - 2], [p[L - 1] for p in z['Ap_pyr']],
                                 [p[L - 2] for p in z['Ap_pyr']], z['B_pyr'][L - 1], z['B_pyr'][L - 2],
                                 z['Bp_init'][L - 2].copy(), z['Bp_init'][L - 1].copy(), z['weights'], 1.0)
    finally:
        ctx.set_option('shard_emulate', 1)
        ctx.set_option('exchange', 0)
        ctx.set_option('prune_min_rows', 524288)


def test_unpruned_levels_replicate_by_default(ctx):
    """Option shard_unpruned (default 0): only levels that run the pruned scan are sharded (the
    unpruned scan of a small DB gains nothing from 1/W of the tiles).  g64 scans
    unpruned: one distance launch per step unless shard_unpruned = 1 (then W on its large levels);
    with every level pruned (prune_min_rows = 1) the large levels shard by default."""
    z = load_e2e('g64')
    _, _, st0 = _run(ctx, z, 2, False, 1, shard_unpruned=0)
    _, _, st1 = _run(ctx, z, 2, False, 1, shard_unpruned=1)
    _, _, st2 = _run(ctx, z, 2, True, 1, shard_unpruned=0)
    assert st0.dist_launches <= st0.steps          # one scan per (non-empty) step
    assert st1.dist_launches > st0.dist_launches and st2.dist_launches > st0.dist_launches


def _run_batch(ctx, z, jobs, W, exchange, prune_all=True):
    """jobs = [(kappa, Bp pyramid)] sharing z's A side: one ia_synthesize_levels call per level
    (every job's replica on every emulated rank, one scan per shard for all jobs' queries)."""
    from ia_amd import _native
    L = z['L']
    S, IM = [dict() for _ in jobs], [dict() for _ in jobs]
    st = _native.Stats()
    ctx.set_option('shard_emulate', W)
    ctx.set_option('exchange', exchange)
    if prune_all:
        ctx.set_option('prune_min_rows', 1)
    try:
        for level in range(1, L):
            specs = [dict(B=z['B_pyr'][level], Bc=z['B_pyr'][level - 1], Bpc=Bp[level - 1], Bp=Bp[level],
                          weights=z['weights'], kappa_factor=1 + 2.0 ** (level - L) * k) for k, Bp in jobs]
            res = ctx.synthesize_levels(z['A_pyr'][level], z['A_pyr'][level - 1], [p[level] for p in z['Ap_pyr']],
                                        [p[level - 1] for p in z['Ap_pyr']], specs, st)
            for j, (s, im) in enumerate(res):
                S[j][level], IM[j][level] = s, im
    finally:
        ctx.set_option('shard_emulate', 1)
        ctx.set_option('exchange', 0)
        ctx.set_option('prune_min_rows', 524288)
    return S, IM, st


@pytest.mark.parametrize('exchange', [0, 1, 2, 3], ids=['allgather', 'peerwrite', 'owner', 'owner_k2s'])
@pytest.mark.parametrize('W', [2, 4, 8])
def test_emulated_shards_batched_jobs_match_reference(ctx, W, exchange):
    """W jobs on the golden g256 run's A side stepped together over a W-way sharded DB (bench.py's
    N > 1 shard mode: every rank scans its shard for all jobs' queries; on the 256^2 level 8 x 86
    queries per step = 22 query tiles, the one-launch two-block presorted scan per shard).  Job 0
    is the reference's own run; every job equals the unsharded batched run.  exchange = 2: job j
    owned by shard j (its gather and merge), its queries published by its K2p and sorted inside
    every shard's scan, records pushed to the owner (ia_internal.h XOLayout); owner_k2s: the same
    with the owner's K2s sort + presorted scans (the path of steps wider than 352 queries)."""
    from test_gpu_batch import _jobs_g32
    z = load_e2e('g256')
    kap = (0.5, 5.0, 25.0, 1.0, 2.0, 10.0, 15.0, 20.0)[:max(W, 2)]
    jb = _jobs_g32(z, kappas=kap)
    ju = [(k, [x.copy() for x in Bp]) for k, Bp in jb]
    ctx.set_option('xo_presort', 1 if exchange == 3 else 0)
    try:
        S, IM, st = _run_batch(ctx, z, jb, W, min(exchange, 2))
    finally:
        ctx.set_option('xo_presort', 0)
    Su, IMu, stu = _run_batch(ctx, z, ju, 1, 0)
    for level in range(1, z['L']):
        assert np.array_equal(S[0][level], z['s'][level]) and np.array_equal(IM[0][level], z['im'][level]), level
        assert np.array_equal(jb[0][1][level], z['Bp_final'][level]), level
        for j in range(len(jb)):
            assert np.array_equal(S[j][level], Su[j][level]) and np.array_equal(IM[j][level], IMu[j][level]), (j, level)
            assert np.array_equal(jb[j][1][level], ju[j][1][level]), (j, level)
    assert st.bound_violations == 0 and st.kappa_ambiguous == 0 and st.pixels == stu.pixels
    assert st.dist_launches > stu.dist_launches   # W shard scans per sharded step


@pytest.mark.parametrize('W,exchange', [(4, 1), (2, 2), (8, 2)])
def test_emulated_shards_batched_1024(ctx, W, exchange):
    """W cfg3 jobs (synth.make_jobs: job 0 = cfg3, others other B images) over a W-way sharded
    1024^2 DB with the peer-write winner exchange (1) or owner-computes steps (2, bench.py's N > 1
    shard mode) == the same jobs batched unsharded, every level."""
    from ia_amd import synth
    jobs = synth.make_jobs(W, size=1024)
    z = {'L': jobs[0].L, 'A_pyr': jobs[0].A_pyr, 'Ap_pyr': jobs[0].Ap_pyr_list, 'B_pyr': jobs[0].B_pyr,
         'weights': jobs[0].weights}
    out = []
    for Wx, ex in ((W, exchange), (1, 0)):
        S, IM, Bps = [], [], []
        from ia_amd import _native
        st = _native.Stats()
        ctx.set_option('shard_emulate', Wx)
        ctx.set_option('exchange', ex)
        Bp = [[x.copy() for x in j.Bp_init] for j in jobs]
        try:
            for level in range(1, z['L']):
                specs = [dict(B=j.B_pyr[level], Bc=j.B_pyr[level - 1], Bpc=Bp[n][level - 1], Bp=Bp[n][level],
                              weights=j.weights, kappa_factor=j.kappa_factor(level)) for n, j in enumerate(jobs)]
                res = ctx.synthesize_levels(z['A_pyr'][level], z['A_pyr'][level - 1], [p[level] for p in z['Ap_pyr']],
                                            [p[level - 1] for p in z['Ap_pyr']], specs, st)
                S.append([r[0] for r in res])
                IM.append([r[1] for r in res])
        finally:
            ctx.set_option('shard_emulate', 1)
            ctx.set_option('exchange', 0)
        out.append((S, IM, Bp, st))
    (S, IM, Bp, st), (Su, IMu, Bpu, stu) = out
    for i in range(len(S)):
        for n in range(W):
            assert np.array_equal(S[i][n], Su[i][n]) and np.array_equal(IM[i][n], IMu[i][n]), (i, n)
    for n in range(W):
        for level in range(1, z['L']):
            assert np.array_equal(Bp[n][level], Bpu[n][level]), (n, level)
    assert st.pruned_levels == W and st.bound_violations == 0


def test_owner_exchange_needs_one_job_per_shard(ctx):
    """exchange = 2 emulated: one job per shard (n_jobs = shard_emulate), else IA_EINVAL."""
    from ia_amd import _native
    from test_gpu_batch import _jobs_g32
    z = load_e2e('g256')
    jb = _jobs_g32(z, kappas=(0.5, 5.0, 25.0))
    with pytest.raises(_native.IAError):
        _run_batch(ctx, z, jb, 2, 2)


@pytest.mark.parametrize('presort', [0, 1], ids=['inkernel', 'k2s'])
def test_owner_shards_with_unequal_tile_counts(ctx, presort):
    """owner-computes shards whose tile counts differ by one across a multiple of 8
    (A 66 x 69 = 4,554 rows -> 143 tiles: shards of 72 and 71 tiles, W = 2).  Every shard's scan
    must use the one chunk count the owners' merges assume (from the smaller shard), else records
    overlap or DB chunks drop out; every level pruned, both jobs == their unsharded batched run."""
    from ia_amd import _native, synth
    jobs = synth.make_jobs(2, size=(66, 69))
    assert (66 * 69 + 31) // 32 == 143
    z = {'L': jobs[0].L, 'A_pyr': jobs[0].A_pyr, 'Ap_pyr': jobs[0].Ap_pyr_list}
    out = []
    ctx.set_option('xo_presort', presort)
    ctx.set_option('prune_min_rows', 1)
    try:
        for Wx, ex in ((2, 2), (1, 0)):
            S, IM = [], []
            st = _native.Stats()
            ctx.set_option('shard_emulate', Wx)
            ctx.set_option('exchange', ex)
            Bp = [[x.copy() for x in j.Bp_init] for j in jobs]
            for level in range(1, z['L']):
                specs = [dict(B=j.B_pyr[level], Bc=j.B_pyr[level - 1], Bpc=Bp[n][level - 1], Bp=Bp[n][level],
                              weights=j.weights, kappa_factor=j.kappa_factor(level)) for n, j in enumerate(jobs)]
                res = ctx.synthesize_levels(z['A_pyr'][level], z['A_pyr'][level - 1], [p[level] for p in z['Ap_pyr']],
                                            [p[level - 1] for p in z['Ap_pyr']], specs, st)
                S.append([r[0] for r in res])
                IM.append([r[1] for r in res])
            out.append((S, IM, Bp, st))
    finally:
        ctx.set_option('shard_emulate', 1)
        ctx.set_option('exchange', 0)
        ctx.set_option('xo_presort', 0)
        ctx.set_option('prune_min_rows', 524288)
    (S, IM, Bp, st), (Su, IMu, Bpu, stu) = out
    for i in range(len(S)):
        for n in range(2):
            assert np.array_equal(S[i][n], Su[i][n]) and np.array_equal(IM[i][n], IMu[i][n]), (i, n)
    for n in range(2):
        for level in range(1, z['L']):
            assert np.array_equal(Bp[n][level], Bpu[n][level]), (n, level)
    assert st.bound_violations == 0 and st.dist_launches > stu.dist_launches
