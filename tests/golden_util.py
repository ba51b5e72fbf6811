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
