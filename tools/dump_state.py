"""Run a synthetic job on the GPU (default options: the product kernels) and save the
synthesised state of the given levels (B' levels, s, im) for offline teacher forcing
(tools/teacher_force.py) and analysis (tools/prune_study.py).  Usage:
  python3 tools/dump_state.py <out.npz> [config|size] [levels...]
config: a name of ia_amd.synth.CONFIGS (cfg3, cfg4, ...) or an integer size (square A = B)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ia_amd  # noqa: F401,E402
from ia_amd import _native, synth  # noqa: E402

out = sys.argv[1]
cfg = sys.argv[2] if len(sys.argv) > 2 else '1024'
kw = dict(size=int(cfg)) if cfg.isdigit() else synth.CONFIGS[cfg][0]
job = synth.make_job(**kw)
levels = [int(x) for x in sys.argv[3:]] or [job.L - 2, job.L - 1]
ctx = _native.Context(0)
Bp = [x.copy() for x in job.Bp_init]
S, IM = {}, {}
st = _native.Stats()
for level in range(1, job.L):
    S[level], IM[level] = ctx.synthesize_level(
        job.A_pyr[level], job.A_pyr[level - 1], [p[level] for p in job.Ap_pyr_list],
        [p[level - 1] for p in job.Ap_pyr_list], job.B_pyr[level], job.B_pyr[level - 1], Bp[level - 1], Bp[level],
        job.weights, job.kappa_factor(level), st)
# B' of a synthesised level is A' at its sources (B'[p] = A'_im[p][s[p]], the merge's writeback),
# so only s (int16) and im (uint8) travel; tools/teacher_force.py rebuilds B' from the job's A'
# pyramid and checks it against the sha1 of the GPU's B' bytes stored here
import hashlib  # noqa: E402
d = {}
for l in sorted(set(levels) | {l - 1 for l in levels if l > 1}):
    assert S[l].max() < 32768 and IM[l].max() < 256
    d['s_%d' % l] = S[l].astype(np.int16)
    d['im_%d' % l] = IM[l].astype(np.uint8)
    d['bpsha_%d' % l] = np.frombuffer(hashlib.sha1(np.ascontiguousarray(Bp[l]).tobytes()).digest(), dtype=np.uint8)
np.savez_compressed(out, size=int(kw['size']) if np.isscalar(kw['size']) else 0, config=cfg, levels=np.array(levels), **d)
print('saved', out, os.path.getsize(out), 'stats', {k: v for k, v in st.as_dict().items()
                                                      if k in ('pixels', 'fallbacks', 'reranked', 'bound_violations',
                                                               'kappa_ambiguous', 'pruned_levels')})
