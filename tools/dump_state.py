"""Run the cfg3 synthetic job on the GPU and save the synthesised state of the finest levels
(B' levels, s, im) for offline analysis (tools/prune_study.py).  Usage:
  python3 tools/dump_state.py <out.npz> [size] [levels...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ia_amd  # noqa: F401,E402
from ia_amd import _native, synth  # noqa: E402

out = sys.argv[1]
size = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
job = synth.make_job(size)
levels = [int(x) for x in sys.argv[3:]] or [job.L - 2, job.L - 1]
ctx = _native.Context(0)
Bp = [x.copy() for x in job.Bp_init]
S, IM = {}, {}
for level in range(1, job.L):
    S[level], IM[level] = ctx.synthesize_level(
        job.A_pyr[level], job.A_pyr[level - 1], [p[level] for p in job.Ap_pyr_list],
        [p[level - 1] for p in job.Ap_pyr_list], job.B_pyr[level], job.B_pyr[level - 1], Bp[level - 1], Bp[level],
        job.weights, job.kappa_factor(level))
d = {}
for l in levels:
    d['Bp_%d' % l] = Bp[l]
    d['Bp_%d' % (l - 1)] = Bp[l - 1]
    d['s_%d' % l] = S[l]
    d['im_%d' % l] = IM[l]
np.savez_compressed(out, size=size, levels=np.array(levels), **d)
print('saved', out, os.path.getsize(out))
