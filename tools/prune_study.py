"""Offline study: how selective would certified bounds be for pruning the exact NN scan?
Uses GPU-synthesised state (tools/dump_state.py) and the oracle's feature functions.
For sampled pixels: U = exact distance of the best coherence candidate (an upper bound on the
NN distance), and the fraction of DB rows a lower bound cannot exclude (bound <= U).
  python3 tools/prune_study.py <state.npz> [level] [n_pixels]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ia_amd import synth  # noqa: E402
from oracle import ia_oracle as O  # noqa: E402

z = np.load(sys.argv[1])
level = int(sys.argv[2]) if len(sys.argv) > 2 else 8
n = int(sys.argv[3]) if len(sys.argv) > 3 else 100
job = synth.make_job(int(z['size']))
As = O.build_db(job.A_pyr, job.Ap_pyr_list, level)
Bf = O.feature_array(job.B_pyr, level, True)
h, w = job.B_pyr[level].shape[:2]
A_h, A_w = job.A_pyr[level].shape[:2]
Bp_f, Bp_sm = z['Bp_%d' % level], z['Bp_%d' % (level - 1)]
s, im = z['s_%d' % level].astype(np.int64), z['im_%d' % level].astype(np.int64)
mu = As.mean(axis=0)
X = As - mu
sub = X[np.random.RandomState(0).choice(len(X), min(len(X), 50000), replace=False)]
_, sv, Vt = np.linalg.svd(sub, full_matrices=False)
print('level', level, 'rows', len(As), 'explained var of PC1..8:', np.round(sv[:8] ** 2 / (sv ** 2).sum(), 3))
P = X @ Vt[:16].T                       # projections on the first 16 PCs
norms = np.sqrt((X * X).sum(axis=1))
rs = np.random.RandomState(1)
pix = rs.randint(w * 3, h * w, n)
stats = []
for qi in pix:
    r, c = divmod(int(qi), w)
    lg = O.state_at(Bp_f, job.Bp_init[level], qi)
    q = O.query_feature(Bf, Bp_sm, lg, r, c, w)
    d = ((As - q) ** 2).sum(axis=1)
    dnn = d.min()
    cand = []
    for rr in range(max(0, r - 2), r + 1):
        for rc in range(max(0, c - 2), min(w, c + 3)):
            ri = rr * w + rc
            if ri >= qi:
                continue
            pr, pc = s[ri, 0] + r - rr, s[ri, 1] + c - rc
            if 0 <= pr < A_h and 0 <= pc < A_w:
                cand.append((A_h * im[ri] + pr) * A_w + pc)
    if not cand:
        continue
    U = d[np.array(cand)].min()
    qc = q - mu
    qp = qc @ Vt[:16].T
    row = {'U/dnn': U / max(dnn, 1e-300), 'ideal': (d <= U).mean()}
    for k in (1, 2, 4, 8, 16):
        lb = ((P[:, :k] - qp[:k]) ** 2).sum(axis=1)
        row['pc%d' % k] = (lb <= U).mean()
    row['norm'] = ((norms - np.sqrt((qc * qc).sum())) ** 2 <= U).mean()
    stats.append(row)
for k in stats[0]:
    v = np.array([x[k] for x in stats])
    print('%-6s mean %.4f median %.4f p90 %.4f max %.4f' % (k, v.mean(), np.median(v), np.percentile(v, 90), v.max()))
