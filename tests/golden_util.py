"""Helpers to read the golden end-to-end fixtures written by oracle/gen_golden.py."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
E2E_CASES = ['g32', 'g24k5', 'rect', 'g64', 'yiq', 'remap', 'rgb3', 'multiap', 'noinit', 'ties']
# round-2 reference runs at larger sizes (oracle/gen_golden.py big_cases; 'lean' fixtures):
# cfg1 = BASELINE config 1's 117x180 YIQ stand-in, g128 / g256 = the bench generator,
# ties128 = piecewise-constant (duplicate DB rows), k25 = kappa 25
BIG_CASES = [c for c in ['cfg1', 'g128', 'ties128', 'k25', 'g256']
             if os.path.exists(os.path.join(GOLDEN, 'e2e_%s.npz' % c))]


def load_e2e(name):
    z = np.load(os.path.join(GOLDEN, 'e2e_%s.npz' % name))
    L = int(z['L'])
    nap = z['Ap'].shape[0]
    nB = len([k for k in z.keys() if k.startswith('Bp0_')])
    d = {k: z[k] for k in z.keys()}
    d['L'] = L
    d['A_pyr'] = [z['A_%d' % l] for l in range(L)]
    d['Ap_pyr'] = [[z['Ap%d_%d' % (j, l)] for l in range(L)] for j in range(nap)]
    d['B_pyr'] = [z['B_%d' % l] for l in range(nB)]
    d['Bp_init'] = [z['Bp0_%d' % l] for l in range(nB)]
    d['Bp_final'] = [z['Bp_%d' % l] for l in range(nB)]
    d['s'] = {l: z['s_%d' % l].astype(np.int64) for l in range(1, L)}
    d['im'] = {l: z['im_%d' % l].astype(np.int64) for l in range(1, L)}
    d['app_ix'] = z['app_ix'].astype(np.int64)
    d['coh'] = z['coh'].astype(np.int64)
    return d


# round 6: reference run at BASELINE config 2's shape (512^2, the finest 5 levels), the size at
# which the product's default path prunes; 'slim' fixture (oracle/gen_golden.py run_case slim=True)
SLIM_CASES = [c for c in ['g512', 'g64slim'] if os.path.exists(os.path.join(GOLDEN, 'e2e_%s.npz' % c))]


def sha1_f64(x):
    import hashlib
    return hashlib.sha1(np.ascontiguousarray(x, dtype=np.float64).tobytes()).hexdigest()


def load_slim(name):
    """A slim fixture: the reference's pyramids, s / im of every level, and the sha1 of every B'
    initialisation / final B' level.  Bp_init is rebuilt with the product's seeded
    initialize_Bp and checked against the reference's hashes here."""
    from ia_amd.img_preprocess import initialize_Bp
    z = np.load(os.path.join(GOLDEN, 'e2e_%s.npz' % name))
    L = int(z['L'])
    nap = int(z['n_ap'])
    d = {'L': L, 'k': float(z['k']), 'weights': z['weights']}
    d['A_pyr'] = [z['A_%d' % l] for l in range(L)]
    d['Ap_pyr'] = [[z['Ap%d_%d' % (j, l)] for l in range(L)] for j in range(nap)]
    d['B_pyr'] = [z['B_%d' % l] for l in range(L)]
    d['sha1'] = dict(zip([str(k) for k in z['sha1_keys']], [str(v) for v in z['sha1_vals']]))
    d['Bp_init'] = initialize_Bp(d['B_pyr'], init_rand=True, seed=int(z['seed']))
    for l in range(L):
        assert sha1_f64(d['Bp_init'][l]) == d['sha1']['Bp0_%d' % l], 'B\' init of level %d differs' % l
    d['s'] = {l: z['s_%d' % l].astype(np.int64) for l in range(1, L)}
    d['im'] = {l: z['im_%d' % l].astype(np.int64) for l in range(1, L)}
    return d
