"""Offline study of a second, in-block filter for the pruned scan (K3p), on GPU-synthesised
state (dump_state.py): of the (DB tile, query tile) blocks that pass the 4-D box test, how many
hold at least one pair whose distance is within the query's bound U' plus a margin E?  A block
with none could skip the two hi/lo correction MFMA products and the top-2 epilogue after the
hi x hi product (its rows cannot be or tie the NN), if E bounds the hi-only error.
  python3 tools/hh_filter_sim.py <state.npz> [level] [steps...]"""
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
xn = np.sqrt((X ** 2).sum(axis=1))
R = xn.max()
sub = X[np.random.RandomState(0).choice(len(X), min(len(X), 50000), replace=False)]
_, _, Vt = np.linalg.svd(sub, full_matrices=False)
U_ = Vt[:4]
P = X @ U_.T
bits = 16
lo, hi = P.min(axis=0), P.max(axis=0)
order = np.argsort(morton([quant(P[:, i], lo[i], hi[i], bits) for i in range(4)], bits), kind='stable')
nt = -(-len(order) // 32)
pad = np.concatenate([order, np.full(nt * 32 - len(order), order[-1])])
Pt = P[pad].reshape(nt, 32, 4)
blo, bhi = Pt.min(axis=1), Pt.max(axis=1)
Xs = X[pad]
print('level %d: %d rows, R = max |a - mu| = %.3f, median |a - mu| = %.3f' % (level, len(X), R, np.median(xn)))
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
    qn = np.sqrt((Q ** 2).sum(axis=1))
    Qp = Q @ U_.T
    qorder = np.argsort(morton([quant(Qp[:, i], lo[i], hi[i], bits) for i in range(4)], bits), kind='stable')
    M = len(Q)
    margins = {'0': lambda a, q: 0.0 * a * q,
               '2^-10*2|a||q|+2^-11|a|^2': lambda a, q: 2.0 ** -10 * 2 * a * q + 2.0 ** -11 * a * a,
               '2^-9*(2|a||q|+|a|^2)': lambda a, q: 2.0 ** -9 * (2 * a * q + a * a),
               '2^-9*(2Rt|q|+Rt^2)+2^-16 (tile max |a|)': None,
               '2^-9*(2R|q|+R^2)': lambda a, q: 2.0 ** -9 * (2 * R * q + R * R) + 0 * a}
    blocks, passing = 0, {k: 0 for k in margins}
    tile_need = np.zeros(nt, bool)
    tile_lo = {k: np.zeros(nt, bool) for k in margins}
    for j in range(-(-M // 32)):
        ids = qorder[j * 32:(j + 1) * 32]
        d = np.maximum(0, np.maximum(blo[None] - Qp[ids, None], Qp[ids, None] - bhi[None]))
        need = ((d ** 2).sum(axis=2) <= Uq[ids, None]).any(axis=0)   # box test, per DB tile
        tiles = np.nonzero(need)[0]
        rows = Xs.reshape(nt, 32, -1)[tiles].reshape(-1, Xs.shape[1])
        rn = xn[pad].reshape(nt, 32)[tiles].reshape(-1)
        d2 = (rows ** 2).sum(axis=1)[:, None] - 2 * rows @ Q[ids].T + (Q[ids] ** 2).sum(axis=1)[None]
        blocks += len(tiles)
        tile_need[tiles] = True
        Rt = np.repeat(rn.reshape(len(tiles), 32).max(axis=1), 32)
        for k, f in margins.items():
            if f is None:
                E = 2.0 ** -9 * (2 * Rt[:, None] * qn[ids][None] + Rt[:, None] ** 2) + 2.0 ** -16
            else:
                E = f(rn[:, None], qn[ids][None])
            hit = (d2 <= Uq[ids][None] + E).reshape(len(tiles), 32, len(ids)).any(axis=(1, 2))
            passing[k] += hit.sum()
            tile_lo[k][tiles[hit]] = True
    print('step %d M %d: %d box-needed blocks (%.3f of all); pass fraction by margin: %s'
          % (step, M, blocks, blocks / (nt * -(-M // 32)),
             ', '.join('%s %.3f' % (k, v / blocks) for k, v in passing.items())))
    print('  median U %.4f, median |q - mu| %.3f' % (np.median(Uq), np.median(qn)))
    print('  DB tiles loaded %.3f; of them needing the lo half: %s' % (tile_need.mean(), ', '.join(
        '%s %.3f' % (k, tile_lo[k].sum() / tile_need.sum()) for k in margins)))
