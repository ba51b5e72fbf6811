"""Host logic of the sweep runner (ia_amd.sweep): a job with n_levels = n uses the finest n levels
of the full pyramid (what compute_gaussian_pyramid(img, 3, n) makes), the coarse-to-fine
batching schedule, kappa factors and pixel counts (BASELINE config 5)."""
import numpy as np

import ia_amd  # noqa: F401
from ia_amd import sweep, synth
from ia_amd.img_preprocess import compute_gaussian_pyramid, initialize_Bp


def test_truncated_pyramid_is_the_finest_levels_of_the_full_one():
    img = synth.smooth(80, 72, 2, 5)
    full = compute_gaussian_pyramid(img, 3)
    for n in range(2, len(full) + 1):
        part = compute_gaussian_pyramid(img, 3, n)
        assert len(part) == n
        for a, b in zip(part, full[-n:]):
            assert np.array_equal(a, b)


def test_sweep_schedule_and_kappa():
    A = synth.smooth(64, 64, 2, 1)
    jobs = [sweep.SweepJob(k, n) for k in (0.5, 25) for n in (2, 4, None)]
    sw = sweep.Sweep(A, [synth.filt(A)], synth.smooth(64, 64, 2, 2), jobs)
    assert sw.Lf == 6 and sw.L == [2, 4, 6, 2, 4, 6]
    sched = sw.schedule(max_batch=4)
    seen = {}
    for f, part in sched:
        assert 1 <= len(part) <= 4
        for j, l in part:
            assert l == f - sw.offset(j) and 1 <= l < sw.L[j]
            assert (j, l) not in seen
            seen[(j, l)] = f
    assert sorted(seen) == sorted((j, l) for j in range(6) for l in range(1, sw.L[j]))
    fs = [f for f, _ in sched]
    assert fs == sorted(fs)                   # coarse to fine: level l-1 of every job is done first
    assert sw.kappa_factor(1, 3) == 1 + 2.0 ** (3 - 4) * 0.5
    assert sw.pixels([0]) == 64 * 64 and sw.pixels([2]) == sum(4 ** i for i in range(2, 7))
    # each job's B' init is initialize_Bp of its own pyramid (draw order of its depth)
    ref = initialize_Bp(sw.B_pyr[sw.offset(1):], True, seed=3)
    assert all(np.array_equal(a, b) for a, b in zip(sw.Bp_init[1], ref))


def test_cfg5_jobs():
    jobs = sweep.cfg5_jobs()
    assert len(jobs) == 64 and {j.n_levels for j in jobs} == set(range(2, 10))
    assert {j.k for j in jobs} == {0.5, 1, 2, 5, 10, 15, 20, 25}


def test_unequal_pyramids_pair_coarse_levels_like_the_reference():
    """image_analogies.py:82-86: max_levels = min(len(A_pyr), len(B_pyr)) and the loop walks levels
    0..max_levels-1 of both coarsest-first lists, i.e. the coarsest levels pair and the deeper
    pyramid's extra fine levels are dropped (with a warning).  'fine' pairs the finest levels."""
    import warnings
    A = synth.smooth(40, 40, 2, 1)
    B = synth.smooth(80, 80, 2, 2)
    Af, Bf = compute_gaussian_pyramid(A, 3), compute_gaussian_pyramid(B, 3)
    assert len(Bf) == len(Af) + 1
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        sw = sweep.Sweep(A, [synth.filt(A)], B, [sweep.SweepJob(0.5)])
    assert any('different sizes' in str(x.message) for x in w)
    assert sw.Lf == len(Af)
    assert all(np.array_equal(a, b) for a, b in zip(sw.B_pyr, Bf[:len(Af)]))
    assert all(np.array_equal(a, b) for a, b in zip(sw.A_pyr, Af))
    fine = sweep.Sweep(A, [synth.filt(A)], B, [sweep.SweepJob(0.5)], level_align='fine')
    assert all(np.array_equal(a, b) for a, b in zip(fine.B_pyr, Bf[1:]))
    assert fine.B_pyr[-1].shape == (80, 80) and sw.B_pyr[-1].shape == (40, 40)
