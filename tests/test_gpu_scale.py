"""GPU parity at sizes the oracle cannot run free (SURVEY §7 hard part 2): the GPU synthesises the
whole job; the oracle's decision functions then re-decide sampled pixels on the GPU's own state
(teacher forcing: B' final for raster-earlier pixels, initial for the rest, s / im final).  Every
sampled decision must match, except at documented near-ties: an NN relative gap < 1e-5 between the
best and second-best DB rows, or a kappa-rule relative margin < 1e-12 (BLAS dot order).
Plus the driver end to end and size-independent invariants of the source maps."""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import ia_amd  # noqa: F401
from golden_util import load_e2e
from oracle import ia_oracle as O

pytestmark = pytest.mark.gpu
TF_THREADS = min(16, os.cpu_count() or 1)   # (the GPU box's CPU share is 16 cores)


def _run_job(ctx, job):
    from ia_amd import _native
    Bp = [x.copy() for x in job.Bp_init]
    S, IM = {}, {}
    st = _native.Stats()
    for level in range(1, job.L):
        S[level], IM[level] = ctx.synthesize_level(
            job.A_pyr[level], job.A_pyr[level - 1], [p[level] for p in job.Ap_pyr_list],
            [p[level - 1] for p in job.Ap_pyr_list], job.B_pyr[level], job.B_pyr[level - 1], Bp[level - 1],
            Bp[level], job.weights, job.kappa_factor(level), st)
    return Bp, S, IM, st


def _teacher_force(job, Bp, S, IM, level, n, seed=0):
    As = O.build_db(job.A_pyr, job.Ap_pyr_list, level)
    Bf = O.feature_array(job.B_pyr, level, True)
    h, w = job.B_pyr[level].shape[:2]
    A_h, A_w = job.A_pyr[level].shape[:2]
    rs = np.random.RandomState(seed)
    pix = np.unique(np.concatenate([rs.randint(0, h * w, n), [0, 1, w - 1, w, h * w - 1]]))
    s, im = S[level].astype(np.int64), IM[level].astype(np.int64)

    def one(qi):
        r, c = divmod(int(qi), w)
        out = O.decide_pixel(As, Bf, Bp[level - 1], Bp[level], job.Bp_init[level], s, im, A_h, A_w, level, job.L,
                             job.k, job.weights, r, c)
        (pr, pc), img = out['choice']
        if (pr, pc, img) != (s[qi, 0], s[qi, 1], im[qi]):
            near = out['app_gap'] < 1e-5 or out.get('kappa_gap', 1.0) < 1e-12
            return (int(qi), near, out['app_gap'], out.get('kappa_gap'))
        return None

    # the oracle's per-pixel decisions are numpy-bound (the exact NN streams the whole DB, the GIL
    # released): threads of this process, no child processes after the GPU was initialised
    with ThreadPoolExecutor(max_workers=TF_THREADS) as ex:
        res = list(ex.map(one, pix))
    return len(pix), [m for m in res if m is not None]


@pytest.mark.parametrize('size,levels,n', [(256, (7, 6), 150)])
def test_teacher_forced_256(ctx, size, levels, n):
    from ia_amd import synth
    job = synth.make_job(size)
    Bp, S, IM, st = _run_job(ctx, job)
    assert st.pixels == job.pixels
    _invariants(job, Bp, S, IM)
    for level in levels:
        npx, mism = _teacher_force(job, Bp, S, IM, level, n, seed=level)
        assert all(near for _, near, _, _ in mism), mism
        assert len(mism) <= max(1, npx // 100), mism


def _invariants(job, Bp, S, IM):
    """size-independent invariants on every level: sources inside A, B' values copied from A'"""
    for level in range(1, job.L):
        s, im = S[level], IM[level]
        A_h, A_w = job.A_pyr[level].shape[:2]
        assert (s[:, 0] >= 0).all() and (s[:, 0] < A_h).all() and (s[:, 1] >= 0).all() and (s[:, 1] < A_w).all()
        assert (im == 0).all()
        assert np.array_equal(Bp[level].ravel(), job.Ap_pyr_list[0][level][s[:, 0], s[:, 1]])


def test_teacher_forced_cfg2(ctx):
    """BASELINE config 2 (512^2, n_levels=5: the kappa factor uses L = 5): every synthesised level
    teacher-forced on 100 sampled pixels."""
    from ia_amd import synth
    job = synth.make_job(**synth.CONFIGS['cfg2'][0])
    assert job.L == 5 and job.B_pyr[-1].shape == (512, 512)
    Bp, S, IM, st = _run_job(ctx, job)
    assert st.pixels == job.pixels and st.bound_violations == 0
    _invariants(job, Bp, S, IM)
    for level in range(1, job.L):
        npx, mism = _teacher_force(job, Bp, S, IM, level, 100, seed=10 + level)
        assert all(near for _, near, _, _ in mism), (level, mism)
        assert len(mism) <= max(1, npx // 100), (level, mism)


def test_teacher_forced_1024_levels_5_to_9(ctx):
    """cfg3 (BASELINE metric config): the full 10-level 1024^2 job (pruned scan on the 1024^2
    level), sampled pixels teacher-forced on each of levels 5..9 (64^2 .. 1024^2): 200 on levels
    5-7, 1,000 on the 512^2 level and 800 on the 1024^2 level (the two pruned-scan levels)."""
    from ia_amd import synth
    job = synth.make_job(1024)
    Bp, S, IM, st = _run_job(ctx, job)
    L = job.L
    _invariants(job, Bp, S, IM)
    for level in range(5, L):
        npx, mism = _teacher_force(job, Bp, S, IM, level, {8: 1000, 9: 800}.get(level, 200), seed=level)
        assert all(near for _, near, _, _ in mism), (level, mism)
        assert len(mism) <= max(1, npx // 100), (level, mism)
    assert st.fallbacks < 0.01 * st.pixels
    assert st.bound_violations == 0 and st.f16_levels == L - 1   # default matcher: split-f16
    assert st.pruned_levels == 1


def test_driver_end_to_end_matches_oracle(tmp_path):
    """image_analogies_main (arrays in place of file names, YIQ path) against the oracle run on
    the same host-side pyramids, and against the reference's own output (PSNR >= 50 dB)."""
    from ia_amd import config as c
    from ia_amd.image_analogies import image_analogies_main, img_setup
    z = load_e2e('yiq')
    c.convert, c.remap_lum, c.init_rand, c.AB_weight, c.k, c.seed = True, False, True, 1, 0.5, int(z['seed'])
    res = image_analogies_main(z['A'], [z['Ap'][0]], z['B'], str(tmp_path) + '/out/', c)
    A_pyr, Ap_pyr_list, B_pyr, Bp0, _, _ = img_setup(z['A'], [z['Ap'][0]], z['B'], str(tmp_path) + '/o2/', c)
    Bp = [x.copy() for x in Bp0]
    S, IM = O.run_all_levels(A_pyr, Ap_pyr_list, B_pyr, Bp, c.k, c.weights)
    for level in range(1, c.max_levels):
        assert np.array_equal(res['s'][level], S[level]) and np.array_equal(res['im'][level], IM[level])
        assert np.array_equal(res['Bp_pyr'][level], Bp[level])
    ref = z['Bp_final'][-1]
    mse = np.mean((res['Bp_pyr'][-1] - ref) ** 2)
    psnr = np.inf if mse == 0 else 10 * np.log10(1.0 / mse)
    assert psnr >= 50, psnr
    assert (tmp_path / 'out' / 'level_4_color.jpg').exists() and (tmp_path / 'out' / 'metadata.txt').exists()


def test_fine_alignment_small_matches_oracle(ctx):
    """level_align='fine' (config.level_align, cfg4's pairing): B 96x96 against A 48x48, B's finest
    level paired with A's finest.  Every level bit-exact against the oracle's restatement of the
    reference loop run on the same aligned pyramids (the loop itself is alignment-agnostic)."""
    from ia_amd import synth
    job = synth.make_job(48, b_size=96, k=25.0, level_align='fine')
    assert job.B_pyr[-1].shape == (96, 96) and job.A_pyr[-1].shape == (48, 48)
    for l in range(job.L):
        assert job.B_pyr[l].shape[0] == 2 * job.A_pyr[l].shape[0]
    Bp, S, IM, st = _run_job(ctx, job)
    Bp_o = [x.copy() for x in job.Bp_init]
    So, IMo = O.run_all_levels(job.A_pyr, job.Ap_pyr_list, job.B_pyr, Bp_o, job.k, job.weights)
    for level in range(1, job.L):
        assert np.array_equal(S[level], So[level]) and np.array_equal(IM[level], IMo[level])
        assert np.array_equal(Bp[level], Bp_o[level])
    assert st.bound_violations == 0 and st.kappa_ambiguous == 0


def test_teacher_forced_cfg4(ctx):
    """BASELINE config 4: B 2048^2 against A 1024^2, kappa 25, level_align='fine' (683 queries per
    step on the 2048^2 level, pruned scan on its 1024^2 DB).  Invariants on every level, 400
    sampled pixels teacher-forced on each of the two finest levels."""
    from ia_amd import synth
    job = synth.make_job(**synth.CONFIGS['cfg4'][0])
    assert job.B_pyr[-1].shape == (2048, 2048) and job.A_pyr[-1].shape == (1024, 1024) and job.k == 25.0
    Bp, S, IM, st = _run_job(ctx, job)
    _invariants(job, Bp, S, IM)
    for level in (job.L - 2, job.L - 1):
        npx, mism = _teacher_force(job, Bp, S, IM, level, 400, seed=40 + level)
        assert all(near for _, near, _, _ in mism), (level, mism)
        assert len(mism) <= max(1, npx // 100), (level, mism)
    assert st.bound_violations == 0 and st.pruned_levels == 1
