"""Offline study of a principal-component partial-distance filter for the pruned scan (K3p), on
GPU-synthesised state (dump_state.py).  For an orthonormal basis u_1..u_k,
sum_{i<=k} (u_i . (a - q))^2 <= |a - q|^2, so a (DB tile, query tile) block none of whose
(row, query) pairs has a k-dimensional partial distance within the query's bound U cannot hold
the exact NN.  A compact projection DB (k coordinates per row) streamed first would leave only
the passing tiles' full rows to load.  Reports, per k: the fraction of the 4-D box-needed blocks
that pass and the fraction of DB tiles that still need their full rows.
  python3 tools/pc_filter_sim.py <state.npz> [level] [steps...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ia_amd import synth  # noqa: E402
from oracle import ia_oracle as O  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prune_tiles_sim_lib import morton, quant  # noqa: E402

z = np.load(sys.argv[1])
level = int(sys.argv[2]) if len(sys.argv) > 2 else 9
job = synth.make_job(int(z['size']))
As = O.build_db(job.A_pyr, job.Ap_pyr_list, level)
Bf = O.feature_array(job.B_pyr, level, True)
h, w = job.B_pyr[level].shape[:2]
A_h, A_w = job.A_pyr[level].shape[:2]
steps = [int(x) for x in sys.argv[3:]] or [w + 3 * (h - 1) // 2]
Bp_f, Bp_sm = z['Bp_%d' % level], z['Bp_%d' % (level - 1)]
s, im = z['s_%d' % level].astype(np.int64), z['im_%d' % level].astype(np.int64)
mu = As.mean(axis=0)
X = As - mu
sub = X[np.random.RandomState(0).choice(len(X), min(len(X), 50000), replace=False)]
_, sv, Vt = np.linalg.svd(sub, full_matrices=False)
ev = sv ** 2 / (sv ** 2).sum()
print('level %d: %d rows; explained variance of the first 4/8/16/24/32 PCs: %s' % (
    level, len(X), ', '.join('%.3f' % ev[:k].sum() for k in (4, 8, 16, 24, 32))))
KS = (4, 8, 12, 16, 24, 32)
Pall = X @ Vt[:max(KS)].T
P = Pall[:, :4]
bits = 16
lo, hi = P.min(axis=0), P.max(axis=0)
order = np.argsort(morton([quant(P[:, i], lo[i], hi[i], bits) for i in range(4)], bits), kind='stable')
nt = -(-len(order) // 32)
pad = np.concatenate([order, np.full(nt * 32 - len(order), order[-1])])
Pt = P[pad].reshape(nt, 32, 4)
blo, bhi = Pt.min(axis=1), Pt.max(axis=1)
Ps = Pall[pad].reshape(nt, 32, -1)
for step in steps:
    r_lo = max(0, -(-(step - w + 1) // 3))
    r_hi = min(h - 1, step // 3)
    qs, us = [], []
    for r in range(r_lo, r_hi + 1):
        c = step - 3 * r
        qi = r * w + c
        lg = O.state_at(Bp_f, job.Bp_init[level], qi)
        q = O.query_feature(Bf, Bp_sm, lg, r, c, w)
        cand = []
        for rr in range(max(0, r - 2), r + 1):
            for rc in range(max(0, c - 2), min(w, c + 3)):
                ri = rr * w + rc
                if ri >= qi:
                    continue
                pr, pc = s[ri, 0] + r - rr, s[ri, 1] + c - rc
                if 0 <= pr < A_h and 0 <= pc < A_w:
                    cand.append((A_h * im[ri] + pr) * A_w + pc)
        U = ((As[np.array(cand)] - q) ** 2).sum(axis=1).min() if cand else np.inf
        qs.append(q)
        us.append(U)
    Q = np.array(qs) - mu
    Uq = np.array(us)
    ok = np.isfinite(Uq)
    Q, Uq = Q[ok], Uq[ok]
    Qall = Q @ Vt[:max(KS)].T
    Qp = Qall[:, :4]
    qorder = np.argsort(morton([quant(Qp[:, i], lo[i], hi[i], bits) for i in range(4)], bits), kind='stable')
    M = len(Q)
    nqt = -(-M // 32)
    blocks = 0
    tile_box = np.zeros(nt, bool)
    passing = {k: 0 for k in KS}
    tile_full = {k: np.zeros(nt, bool) for k in KS}
    rows_pass = {k: 0 for k in KS}
    for j in range(nqt):
        ids = qorder[j * 32:(j + 1) * 32]
        d = np.maximum(0, np.maximum(blo[None] - Qp[ids, None], Qp[ids, None] - bhi[None]))
        need = ((d ** 2).sum(axis=2) <= Uq[ids, None]).any(axis=0)
        tiles = np.nonzero(need)[0]
        blocks += len(tiles)
        tile_box[tiles] = True
        U1 = Uq[ids] * (1 + 2.0 ** -10)
        for k in KS:
            A = Ps[tiles, :, :k].reshape(-1, k)
            Qk = Qall[ids, :k]
            d2 = (A ** 2).sum(axis=1)[:, None] - 2 * A @ Qk.T + (Qk ** 2).sum(axis=1)[None]
            hitp = d2 <= U1[None]
            rows_pass[k] += hitp.sum()
            hit = hitp.reshape(len(tiles), 32, len(ids)).any(axis=(1, 2))
            passing[k] += hit.sum()
            tile_full[k][tiles[hit]] = True
    print('step %d M %d: box-needed blocks %.3f of all, DB tiles touched by the box test %.3f' % (
        step, M, blocks / (nt * nqt), tile_box.mean()))
    for k in KS:
        print('  k=%2d: blocks passing %.3f of box-needed, DB tiles needing full rows %.3f, '
              '(row, query) pairs passing per query %.1f' % (k, passing[k] / blocks, tile_full[k].mean(),
                                                               rows_pass[k] / M))
