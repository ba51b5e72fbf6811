"""Batched levels (ia_synthesize_levels) and parameter sweeps (ia_amd.sweep, BASELINE config 5,
multi_script.py:13-32): several jobs sharing the A side step through one wavefront together -
one gather, one distance scan and one merge per step for all of them - and every job's B', s
and im must be bit-identical to running it alone (and, for the golden job, to the reference)."""
import numpy as np
import pytest
import torch  # noqa: F401  (before libia loads: torch's HIP runtime must be the process's first)

from golden_util import load_e2e

pytestmark = pytest.mark.gpu


def _jobs_g32(z, kappas=(0.5, 5.0, 25.0, 1.0)):
    """the golden g32 job (k = 0.5, the reference's B' init) + variants: other kappas and B' inits"""
    from ia_amd.img_preprocess import initialize_Bp
    out = []
    for n, k in enumerate(kappas):
        Bp = [x.copy() for x in z['Bp_init']] if n == 0 else initialize_Bp(z['B_pyr'], True, seed=100 + n)
        out.append((k, Bp))
    return out


def _run(ctx, z, jobs, batched):
    from ia_amd import _native
    L = z['L']
    S, IM = [dict() for _ in jobs], [dict() for _ in jobs]
    st = _native.Stats()
    for level in range(1, L):
        specs = [dict(B=z['B_pyr'][level], Bc=z['B_pyr'][level - 1], Bpc=Bp[level - 1], Bp=Bp[level],
                      weights=z['weights'], kappa_factor=1 + 2.0 ** (level - L) * k) for k, Bp in jobs]
        if batched:
            res = ctx.synthesize_levels(z['A_pyr'][level], z['A_pyr'][level - 1], [p[level] for p in z['Ap_pyr']],
                                        [p[level - 1] for p in z['Ap_pyr']], specs, st)
        else:
            res = [ctx.synthesize_levels(z['A_pyr'][level], z['A_pyr'][level - 1], [p[level] for p in z['Ap_pyr']],
                                         [p[level - 1] for p in z['Ap_pyr']], [sp], st)[0] for sp in specs]
        for j, (s, im) in enumerate(res):
            S[j][level], IM[j][level] = s, im
    return S, IM, st


@pytest.mark.parametrize('mode', ['default', 'pruned', 'f32', 'fuse_unpruned'])
@pytest.mark.parametrize('name', ['g32', 'multiap', 'ties'])
def test_batched_levels_match_separate_and_reference(ctx, name, mode):
    """pruned: every level pruned, the batched steps run the fused merge + gather per job
    (k_merge_gather with one handoff row set per job); fuse_unpruned: the fused launch on the
    unpruned levels too"""
    from ia_amd import _native
    z = load_e2e(name)
    if mode == 'pruned':
        ctx.set_option('prune_min_rows', 1)
    if mode == 'fuse_unpruned':
        ctx.set_option('fuse_unpruned', 1)
    if mode == 'f32':
        ctx.set_option('matcher', _native.IA_MATCH_F32)
    try:
        jb = _jobs_g32(z)
        js = [(k, [x.copy() for x in Bp]) for k, Bp in jb]
        Sb, IMb, stb = _run(ctx, z, jb, True)
        Ss, IMs, sts = _run(ctx, z, js, False)
    finally:
        ctx.set_option('prune_min_rows', 524288)
        ctx.set_option('matcher', _native.IA_MATCH_F16X3)
        ctx.set_option('fuse_unpruned', 0)
    for j in range(len(jb)):
        for level in range(1, z['L']):
            assert np.array_equal(Sb[j][level], Ss[j][level]) and np.array_equal(IMb[j][level], IMs[j][level])
            assert np.array_equal(jb[j][1][level], js[j][1][level])
    for level in range(1, z['L']):   # job 0 is the reference's own run
        assert np.array_equal(Sb[0][level], z['s'][level]) and np.array_equal(IMb[0][level], z['im'][level])
        assert np.array_equal(jb[0][1][level], z['Bp_final'][level])
    assert stb.pixels == sts.pixels and stb.coherence_wins == sts.coherence_wins
    assert stb.bound_violations == 0 and stb.kappa_ambiguous == 0
    if mode == 'pruned':
        assert stb.pruned_levels == len(jb) * (z['L'] - 1)


@pytest.mark.parametrize('variant', [20, 22, 24, 25])
def test_batched_512_pruned_wide_step(ctx, variant):
    """3 jobs on a 512^2 level with the pruned scan forced: 513 queries per step in one scan (the
    separate runs sort 171 per step) - a different kernel path, the same decisions.  The wide
    steps run the presorted form 21 (under 20, 22 and 24) or 25 (forced)."""
    from ia_amd import synth
    job = synth.make_job(512, n_levels=3)
    ctx.set_option('prune_min_rows', 1)
    ctx.set_option('k3p_variant', variant)
    try:
        z = {'L': job.L, 'A_pyr': job.A_pyr, 'Ap_pyr': job.Ap_pyr_list, 'B_pyr': job.B_pyr, 'weights': job.weights,
             'Bp_init': job.Bp_init}
        jb = _jobs_g32(z, kappas=(0.5, 5.0, 25.0))
        js = [(k, [x.copy() for x in Bp]) for k, Bp in jb]
        Sb, IMb, stb = _run(ctx, z, jb, True)
        Ss, IMs, sts = _run(ctx, z, js, False)
    finally:
        ctx.set_option('prune_min_rows', 524288)
        ctx.set_option('k3p_variant', 24)
    for j in range(len(jb)):
        for level in range(1, job.L):
            assert np.array_equal(Sb[j][level], Ss[j][level]) and np.array_equal(IMb[j][level], IMs[j][level])
            assert np.array_equal(jb[j][1][level], js[j][1][level])
    assert stb.pruned_levels == 3 * (job.L - 1) and stb.bound_violations == 0


def test_sweep_batched_equals_sequential_and_oracle(ctx):
    """A 6-job mini sweep (kappa x pyramid depth, multi_script-style) on 96x96 images: batched ==
    one job at a time, and one job against the oracle's restatement of the reference loop."""
    from ia_amd import sweep, synth
    from oracle import ia_oracle as O
    A = synth.smooth(96, 96, 2, 1)
    Ap = synth.filt(A)
    B = synth.smooth(96, 96, 2, 2)
    jobs = [sweep.SweepJob(k, n, seed=3 + i) for i, (k, n) in enumerate([(0.5, 3), (5, 3), (25, 3), (0.5, 5),
                                                                          (5, 5), (2, None)])]
    sw = sweep.Sweep(A, [Ap], B, jobs)
    rb = sw.run(ctx, batched=True)
    rs = sw.run(ctx, batched=False)
    for j in range(len(jobs)):
        Bpb, Sb, IMb = rb[j]
        Bps, Ss, IMs = rs[j]
        assert sorted(Sb) == list(range(1, sw.L[j]))
        for level in Sb:
            assert np.array_equal(Sb[level], Ss[level]) and np.array_equal(IMb[level], IMs[level])
            assert np.array_equal(Bpb[level], Bps[level])
    j = 4   # k = 5, 5 levels
    off = sw.offset(j)
    Bp = [x.copy() for x in sw.Bp_init[j]]
    S, IM = O.run_all_levels(sw.A_pyr[off:], [p[off:] for p in sw.Ap_pyr_list], sw.B_pyr[off:], Bp, jobs[j].k,
                             sw.weights)
    for level in range(1, sw.L[j]):
        assert np.array_equal(rb[j][1][level], S[level]) and np.array_equal(rb[j][2][level], IM[level])
        assert np.array_equal(rb[j][0][level], Bp[level])


def test_device_sweep_two_streams_equals_one(ctx):
    """DeviceSweep.run over two contexts (HIP streams, one host thread each; bench.py --streams 2):
    every job's B', s and im bit-identical to the one-context run, stats summed."""
    from ia_amd import _native, sweep, synth
    A = synth.smooth(96, 96, 2, 1)
    jobs = [sweep.SweepJob(k, n, seed=5 + i) for i, (k, n) in enumerate([(0.5, 3), (5, 4), (25, 5), (1, None), (2, 3)])]
    sw = sweep.Sweep(A, [synth.filt(A)], synth.smooth(96, 96, 2, 2), jobs)
    dev = torch.device('cuda', 0)
    ds = sweep.DeviceSweep(sw, range(len(jobs)), torch, dev)
    st1, st2 = _native.Stats(), _native.Stats()
    ds.run(ctx, st1)
    one = {j: ([x.cpu().numpy() for x in ds.Bp[j]], [x.cpu().numpy() for x in ds.S[j]], [x.cpu().numpy() for x in ds.IM[j]])
           for j in range(len(jobs))}
    ctx2 = _native.Context(0)
    ds.run([ctx, ctx2], st2)
    torch.cuda.synchronize()
    for j in range(len(jobs)):
        for level in range(1, sw.L[j]):
            assert np.array_equal(ds.Bp[j][level].cpu().numpy(), one[j][0][level])
            assert np.array_equal(ds.S[j][level].cpu().numpy(), one[j][1][level])
            assert np.array_equal(ds.IM[j][level].cpu().numpy(), one[j][2][level])
    assert st2.pixels == st1.pixels and st2.coherence_wins == st1.coherence_wins and st2.bound_violations == 0


@pytest.mark.parametrize('mode', ['unpruned', 'pruned', 'pruned_seq', 'pruned_v20', 'pruned_v25'])
def test_batched_g256_wide_steps_match_reference(ctx, mode):
    """8 jobs on the golden g256 run's A side: job 0 is the reference's own
    run, jobs 1..7 other kappas and B' seeds.  On the 256^2 level a step holds 8 x 86 = 688
    queries = 22 query tiles, above one launch's 11 (ia_k3h_qtmax) and the in-kernel sort's 512:
      unpruned: the split-f16 scan in two query blocks per step (nqb = 2);
      pruned: prune_min_rows = 1, the presorted wide-step path K2s + v21 as ONE launch of
        2 query blocks x 128 DB chunks (k3p_blocks = 1, the default);
      pruned_seq: the same as one launch per query block (k3p_blocks = 0);
      pruned_v20: the same kernels under option k3p_variant 20;
      pruned_v25: the two-pass scan's presorted form.
    Job 0 must reproduce the reference's s, im and B' on every level; every job must equal its
    own separate run (86-query steps: a single launch, the in-kernel sort)."""
    z = load_e2e('g256')
    if mode != 'unpruned':
        ctx.set_option('prune_min_rows', 1)
    if mode in ('pruned_v20', 'pruned_v25'):
        ctx.set_option('k3p_variant', int(mode[-2:]))
    if mode == 'pruned_seq':
        ctx.set_option('k3p_blocks', 0)
    try:
        jb = _jobs_g32(z, kappas=(0.5, 5.0, 25.0, 1.0, 2.0, 10.0, 15.0, 20.0))
        js = [(k, [x.copy() for x in Bp]) for k, Bp in jb]
        Sb, IMb, stb = _run(ctx, z, jb, True)
        Ss, IMs, sts = _run(ctx, z, js, False)
    finally:
        ctx.set_option('prune_min_rows', 524288)
        ctx.set_option('k3p_variant', 24)
        ctx.set_option('k3p_blocks', 1)
    h, w = z['B_pyr'][-1].shape
    assert 8 * min(h, (w + 2) // 3) > 512
    for level in range(1, z['L']):   # job 0 is the reference's own run
        assert np.array_equal(Sb[0][level], z['s'][level]) and np.array_equal(IMb[0][level], z['im'][level])
        assert np.array_equal(jb[0][1][level], z['Bp_final'][level])
    for j in range(len(jb)):
        for level in range(1, z['L']):
            assert np.array_equal(Sb[j][level], Ss[j][level]) and np.array_equal(IMb[j][level], IMs[j][level])
            assert np.array_equal(jb[j][1][level], js[j][1][level])
    assert stb.pixels == sts.pixels and stb.coherence_wins == sts.coherence_wins
    assert stb.bound_violations == 0 and stb.kappa_ambiguous == 0
    if mode != 'unpruned':
        assert stb.pruned_levels == 8 * (z['L'] - 1)
    # two query blocks on the 256^2 level: more scan launches than steps, except in the pruned
    # scan's one-launch form (one launch per step, twice the box-needed tile visits)
    if mode in ('unpruned', 'pruned_seq'):
        assert stb.dist_launches > stb.steps
    else:
        assert stb.dist_launches <= stb.steps


def test_cfg5_sweep_full_size(ctx):
    """BASELINE config 5 at its own size (multi_script.py:19-32): the 64-job
    kappa x depth sweep (sweep.cfg5_jobs) on 512^2 images, device-resident, batched 16 jobs per
    level call over three contexts (HIP streams + host threads, bench.py --streams 3).  Every job
    must equal the one-job-at-a-time run (the reference's order); the deepest kappa-25 job is
    teacher-forced on >= 50 pixels of every level against the oracle."""
    from ia_amd import _native, sweep, synth
    from test_gpu_scale import _invariants, _teacher_force
    n = synth.CONFIGS['cfg5'][0]['size']
    A = synth.smooth(n, n, 2, 1)
    sw = sweep.Sweep(A, [synth.filt(A)], synth.smooth(n, n, 2, 2), sweep.cfg5_jobs())
    assert len(sw.jobs) == 64 and sw.B_pyr[-1].shape == (512, 512)
    dev = torch.device('cuda', 0)
    ds = sweep.DeviceSweep(sw, range(len(sw.jobs)), torch, dev)
    ctxs = [ctx, _native.Context(0), _native.Context(0)]
    stb = _native.Stats()
    ds.run(ctxs, stb, batched=True, max_batch=16)
    torch.cuda.synchronize()
    assert stb.pixels == sw.pixels() and stb.bound_violations == 0 and stb.kappa_ambiguous == 0
    sts = _native.Stats()
    seq = sw.run(ctx, batched=False, stats=sts)
    assert sts.pixels == stb.pixels and sts.coherence_wins == stb.coherence_wins
    for j in range(len(sw.jobs)):
        Bps, Ss, IMs = seq[j]
        for level in range(1, sw.L[j]):
            assert np.array_equal(ds.S[j][level].cpu().numpy(), Ss[level]), (j, level)
            assert np.array_equal(ds.IM[j][level].cpu().numpy(), IMs[level]), (j, level)
            assert np.array_equal(ds.Bp[j][level].cpu().numpy(), Bps[level]), (j, level)
    deep = max(j for j in range(len(sw.jobs)) if sw.L[j] == max(sw.L) and sw.jobs[j].k == 25)
    off = sw.offset(deep)
    job = synth.Job(sw.A_pyr[off:], [p[off:] for p in sw.Ap_pyr_list], sw.B_pyr[off:], sw.Bp_init[deep],
                    sw.jobs[deep].k, sw.weights)
    Bp, S, IM = seq[deep]
    _invariants(job, Bp, S, IM)
    for level in range(1, job.L):
        n_b = int(np.prod(job.B_pyr[level].shape[:2]))
        npx, mism = _teacher_force(job, Bp, S, IM, level, 60 if n_b > 1024 else 8 * n_b, seed=50 + level)
        assert npx >= min(50, n_b), (level, npx)
        assert all(near for _, near, _, _ in mism), (level, mism)
        assert len(mism) <= max(1, npx // 100), (level, mism)
    for c in ctxs[1:]:
        c.close()


def test_cfg5_pruned_batches_fit_the_chain_budget(ctx):
    """cfg5 with its 512^2 finest levels pruned (prune_min_rows 262,144): 16-job batches put
    16 x 171 = 2,736 queries in a step, and three contexts run such levels at once.  Fused
    merge + gather launches that many waves wide could stall on each other's row handoffs (every
    resident slot held by a wave whose predecessor row is not dispatched); the process-wide
    chained-wave budget (ia_capi.cpp g_chain_waves) makes those levels run separate launches.
    The run must finish and equal the unpruned batched run bit for bit."""
    from ia_amd import _native, sweep, synth
    n = synth.CONFIGS['cfg5'][0]['size']
    A = synth.smooth(n, n, 2, 1)
    sw = sweep.Sweep(A, [synth.filt(A)], synth.smooth(n, n, 2, 2), sweep.cfg5_jobs())
    dev = torch.device('cuda', 0)
    ctxs = [ctx, _native.Context(0), _native.Context(0)]
    try:
        ref = sweep.DeviceSweep(sw, range(len(sw.jobs)), torch, dev)
        ref.run(ctxs, _native.Stats(), batched=True, max_batch=16)
        for c in ctxs:
            c.set_option('prune_min_rows', 262144)
        ds = sweep.DeviceSweep(sw, range(len(sw.jobs)), torch, dev)
        st = _native.Stats()
        ds.run(ctxs, st, batched=True, max_batch=16)
        torch.cuda.synchronize()
    finally:
        ctx.set_option('prune_min_rows', 524288)
        for c in ctxs[1:]:
            c.close()
    assert st.pruned_levels > 0 and st.bound_violations == 0
    for j in range(len(sw.jobs)):
        for level in range(1, sw.L[j]):
            assert np.array_equal(ds.S[j][level].cpu().numpy(), ref.S[j][level].cpu().numpy()), (j, level)
            assert np.array_equal(ds.IM[j][level].cpu().numpy(), ref.IM[j][level].cpu().numpy()), (j, level)
            assert np.array_equal(ds.Bp[j][level].cpu().numpy(), ref.Bp[j][level].cpu().numpy()), (j, level)
