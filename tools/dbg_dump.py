import sys, os
sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
import numpy as np
import ia_amd
from ia_amd import _native
from golden_util import load_e2e
z = load_e2e('g32')
ctx = _native.Context(0)
L, k = z['L'], float(z['k'])
Bp = [x.copy() for x in z['Bp_init']]
out = {}
for level in range(1, L):
    kf = 1 + (2 ** (level - L)) * k
    dbg = {}
    s, im = ctx.synthesize_level(z['A_pyr'][level], z['A_pyr'][level - 1], [p[level] for p in z['Ap_pyr']],
                                 [p[level - 1] for p in z['Ap_pyr']], z['B_pyr'][level], z['B_pyr'][level - 1],
                                 Bp[level - 1], Bp[level], z['weights'], kf, debug=dbg)
    out['src_%d' % level] = dbg['src']; out['dist_%d' % level] = dbg['dist']
os.makedirs('gpurun_out', exist_ok=True)
np.savez('gpurun_out/dbg_g32.npz', **out)
print('ok')
