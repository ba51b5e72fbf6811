"""Level pipelining (include/ia.h ia_pipeline_depend, ia_amd.pipeline): levels
rotate over two (or four, the finest level's stream at high priority) contexts run from one host
thread each, each step of level l + 1 waiting only
for the steps of level l it reads.  Every level's s, im and B' must equal the sequential run's
(and the reference's, for golden cases) bit for bit."""
import numpy as np
import pytest
import torch

from golden_util import BIG_CASES, load_e2e

pytestmark = pytest.mark.gpu


def _device_job(z, dev):
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).to(dev)
    L = z['L']
    d = dict(A=[t(x) for x in z['A_pyr']], Ap=[t(np.stack([p[l] for p in z['Ap_pyr']])) for l in range(L)],
             B=[t(x) for x in z['B_pyr']], Bp=[t(x) for x in z['Bp_init']], W=t(z['weights']))
    d['S'] = [torch.empty((int(np.prod(x.shape[:2])), 2), dtype=torch.int32, device=dev) for x in z['B_pyr']]
    d['IM'] = [torch.empty(int(np.prod(x.shape[:2])), dtype=torch.int32, device=dev) for x in z['B_pyr']]
    return d


def _level_fn(z, d):
    L, k = z['L'], float(z['k'])
    ch = 1 if z['A_pyr'][0].ndim == 2 else z['A_pyr'][0].shape[2]

    def level(ctx, l, st):
        ptrs = dict(A=d['A'][l].data_ptr(), Ac=d['A'][l - 1].data_ptr(), Ap=d['Ap'][l].data_ptr(),
                    Apc=d['Ap'][l - 1].data_ptr(), B=d['B'][l].data_ptr(), Bc=d['B'][l - 1].data_ptr(),
                    Bpc=d['Bp'][l - 1].data_ptr(), Bp=d['Bp'][l].data_ptr(), weights=d['W'].data_ptr(),
                    s_out=d['S'][l].data_ptr(), im_out=d['IM'][l].data_ptr())
        ctx.synthesize_level_device(ch, len(z['Ap_pyr']), d['A'][l].shape[:2], d['B'][l].shape[:2], ptrs,
                                    1 + 2.0 ** (l - L) * k, st)
    return level


def _run(ctxs, z, pipelined, prune_all=False):
    from ia_amd import _native
    from ia_amd.pipeline import run_levels_pipelined
    dev = torch.device('cuda', 0)
    d = _device_job(z, dev)
    for c in ctxs:
        c.set_option('prune_min_rows', 1 if prune_all else 524288)
    st = _native.Stats()
    fn = _level_fn(z, d)
    try:
        if pipelined:
            run_levels_pipelined(fn, ctxs, z['L'], st)
        else:
            for l in range(1, z['L']):
                fn(ctxs[0], l, st)
        torch.cuda.synchronize()
    finally:
        for c in ctxs:
            c.set_option('prune_min_rows', 524288)
    return ([d['S'][l].cpu().numpy() for l in range(z['L'])], [d['IM'][l].cpu().numpy() for l in range(z['L'])],
            [d['Bp'][l].cpu().numpy() for l in range(z['L'])], st)


@pytest.fixture(scope='module')
def ctx2():
    from ia_amd import _native
    c = _native.Context(0)
    yield c
    c.close()


@pytest.fixture(scope='module')
def ctx4():
    """four contexts as bench.py --pipe-ctx 4 --pipe-priority 1 makes them"""
    from ia_amd import _native
    cs = [_native.Context(0) for _ in range(4)]
    cs[0].set_option('stream_priority', 1)
    for c in cs[1:]:
        c.set_option('stream_priority', 2)
    yield cs
    for c in cs:
        c.close()


@pytest.mark.parametrize('nctx', [2, 4])
@pytest.mark.parametrize('prune_all', [False, True], ids=['default', 'pruned'])
@pytest.mark.parametrize('name', ['g64', 'k25', 'ties128'] + [c for c in ('g256',) if c in BIG_CASES])
def test_pipelined_levels_match_reference(ctx, ctx2, ctx4, name, prune_all, nctx):
    z = load_e2e(name)
    S, IM, Bp, st = _run([ctx, ctx2] if nctx == 2 else ctx4, z, True, prune_all)
    for l in range(1, z['L']):
        assert np.array_equal(S[l], z['s'][l]) and np.array_equal(IM[l], z['im'][l]), l
        assert np.array_equal(Bp[l], z['Bp_final'][l]), l
    assert st.bound_violations == 0 and st.pixels == sum(int(np.prod(z['B_pyr'][l].shape[:2])) for l in range(1, z['L']))


@pytest.mark.parametrize('nctx', [2, 3, 4])
def test_pipelined_cfg3_matches_sequential(ctx, ctx2, ctx4, nctx):
    """cfg3 (1024^2, 10 levels: the pruned 1024^2 level overlapping the 512^2 one)"""
    from ia_amd import synth
    job = synth.make_job(1024)
    z = {'L': job.L, 'k': job.k, 'A_pyr': job.A_pyr, 'Ap_pyr': job.Ap_pyr_list, 'B_pyr': job.B_pyr,
         'Bp_init': job.Bp_init, 'weights': job.weights}
    S1, IM1, Bp1, _ = _run([ctx], z, False)
    S2, IM2, Bp2, st = _run([ctx, ctx2] if nctx == 2 else ctx4[:nctx], z, True)
    for l in range(1, job.L):
        assert np.array_equal(S1[l], S2[l]) and np.array_equal(IM1[l], IM2[l]) and np.array_equal(Bp1[l], Bp2[l]), l
    assert st.pruned_levels == 1 and st.bound_violations == 0
