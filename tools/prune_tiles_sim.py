"""Offline simulation of a tile-granular pruned K3 on GPU-synthesised state (dump_state.py):
DB rows sorted by a Morton key over the first NPC principal components into 32-row tiles (PC
boxes per tile); the queries of one wavefront step sorted the same way into 32-query tiles;
U = exact distance of each query's best coherence candidate.  Reports the fraction of
(DB tile, query tile) pairs whose box lower bound cannot exclude every query of the query tile
(MFMA work left) and the fraction of DB tiles loaded at all (HBM bytes left).
  python3 tools/prune_tiles_sim.py <state.npz> [level] [npc] [step]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ia_amd import synth  # noqa: E402
from oracle import ia_oracle as O  # noqa: E402


def morton(cols, bits):
    """interleave the bits of k quantised columns (each in [0, 2^bits))"""
    key = np.zeros(len(cols[0]), dtype=np.uint64)
    for b in range(bits - 1, -1, -1):
        for c in cols:
            key = (key << np.uint64(1)) | ((c >> np.uint64(b)) & np.uint64(1))
    return key


def quant(p, lo, hi, bits):
    return np.clip(((p - lo) / (hi - lo) * (2 ** bits - 1)).astype(np.int64), 0, 2 ** bits - 1).astype(np.uint64)


z = np.load(sys.argv[1])
level = int(sys.argv[2]) if len(sys.argv) > 2 else 9
npc = int(sys.argv[3]) if len(sys.argv) > 3 else 4
job = synth.make_job(int(z['size']))
As = O.build_db(job.A_pyr, job.Ap_pyr_list, level)
Bf = O.feature_array(job.B_pyr, level, True)
h, w = job.B_pyr[level].shape[:2]
A_h, A_w = job.A_pyr[level].shape[:2]
step = int(sys.argv[4]) if len(sys.argv) > 4 else w + 3 * (h - 1) // 2
Bp_f, Bp_sm = z['Bp_%d' % level], z['Bp_%d' % (level - 1)]
s, im = z['s_%d' % level].astype(np.int64), z['im_%d' % level].astype(np.int64)
mu = As.mean(axis=0)
X = As - mu
sub = X[np.random.RandomState(0).choice(len(X), min(len(X), 50000), replace=False)]
_, _, Vt = np.linalg.svd(sub, full_matrices=False)
U_ = Vt[:npc]
P = X @ U_.T
bits = 64 // npc if npc > 1 else 32
bits = min(bits, 16)
lo, hi = P.min(axis=0), P.max(axis=0)
key = morton([quant(P[:, i], lo[i], hi[i], bits) for i in range(npc)], bits)
order = np.argsort(key, kind='stable')
nt = -(-len(order) // 32)
TR = int(os.environ.get("TR", 32)); TQ = int(os.environ.get("TQ", 32)); nt = -(-len(order) // TR)
pad = np.concatenate([order, np.full(nt * TR - len(order), order[-1])])
Pt = P[pad].reshape(nt, TR, npc)
blo, bhi = Pt.min(axis=1), Pt.max(axis=1)           # tile boxes (nt, npc)

# the queries of wavefront step `step`: pixels (r, step - 3r)
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
Q = np.array(qs)
Uq = np.array(us)
Qp = (Q - mu) @ U_.T
M = len(Q)
qkey = morton([quant(Qp[:, i], lo[i], hi[i], bits) for i in range(npc)], bits)
for label, qorder in (('raster', np.arange(M)), ('sorted', np.argsort(qkey, kind='stable'))):
    need = np.zeros((nt,), dtype=bool)
    pairs = 0
    nqt = -(-M // TQ)
    for j in range(nqt):
        ids = qorder[j * TQ:(j + 1) * TQ]
        d = np.maximum(0, np.maximum(blo[None, :, :] - Qp[ids, None, :], Qp[ids, None, :] - bhi[None, :, :]))
        lb = (d ** 2).sum(axis=2)                      # (32, nt)
        tile_need = (lb <= Uq[ids, None]).any(axis=0)
        pairs += tile_need.sum()
        need |= tile_need
    print('level %d npc %d step %d M %d %s: MFMA pairs left %.4f  DB tiles loaded %.4f' %
          (level, npc, step, M, label, pairs / (nqt * nt), need.mean()))
# per-query row-level reference (no tiles)
lbr = []
for k in range(M):
    lbq = ((P - Qp[k]) ** 2).sum(axis=1)
    lbr.append((lbq <= Uq[k]).mean())
print('row-level survivors mean %.4f' % np.mean(lbr))
