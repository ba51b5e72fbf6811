"""How much a tighter per-query bound U would shrink the pruned scan's work:
on GPU-synthesised state (tools/dump_state.py, s / im form), for one wavefront step of the
finest level, the fraction of DB tiles the step's sorted query tiles need (the union the scan
streams) and of (DB tile, query tile) pairs, with U = the best coherence candidate's exact
distance (K2p's bound today) and with U = f x the exact NN distance (f = 1, 1.07, 1.2): what
any tighter bound could reach.  Test infrastructure (uses the oracle's feature code).
Also two candidate sources K2p could add to U: every causal neighbour's exact NN row, shifted by the
neighbour's offset (the coherence rule applied to NN picks the kappa rule overruled), and the
coarser level's pick upsampled (2 s + (r mod 2, c mod 2)).
  python3 tools/prune_u_study.py <state.npz> [step]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
from oracle import ia_oracle as O  # noqa: E402
from teacher_force import _job, rebuild_bp  # noqa: E402
from prune_tiles_sim_lib import morton, quant  # noqa: E402

z = np.load(sys.argv[1])
cfg = str(z['config'])
job = _job(cfg)
level = int(max(z['levels']))
As = O.build_db(job.A_pyr, job.Ap_pyr_list, level)
Bf = O.feature_array(job.B_pyr, level, True)
h, w = job.B_pyr[level].shape[:2]
A_h, A_w = job.A_pyr[level].shape[:2]
step = int(sys.argv[2]) if len(sys.argv) > 2 else w + 3 * (h - 1) // 2
Bp_f, Bp_sm = rebuild_bp(job, z, level), rebuild_bp(job, z, level - 1)
s, im = z['s_%d' % level].astype(np.int64), z['im_%d' % level].astype(np.int64)
npc = 4
mu = As.mean(axis=0)
X = As - mu
sub = X[np.random.RandomState(0).choice(len(X), min(len(X), 50000), replace=False)]
_, _, Vt = np.linalg.svd(sub, full_matrices=False)
U_ = Vt[:npc]
P = X @ U_.T
bits = 16
lo, hi = P.min(axis=0), P.max(axis=0)
order = np.argsort(morton([quant(P[:, i], lo[i], hi[i], bits) for i in range(npc)], bits), kind='stable')
nt = -(-len(order) // 32)
pad = np.concatenate([order, np.full(nt * 32 - len(order), order[-1])])
Pt = P[pad].reshape(nt, 32, npc)
blo, bhi = Pt.min(axis=1), Pt.max(axis=1)
r_lo, r_hi = max(0, -(-(step - w + 1) // 3)), min(h - 1, step // 3)
qs, us = [], []
for r in range(r_lo, r_hi + 1):
    c = step - 3 * r
    qi = r * w + c
    q = O.query_feature(Bf, Bp_sm, O.state_at(Bp_f, job.Bp_init[level], qi), r, c, w)
    cand = []
    for rr in range(max(0, r - 2), r + 1):
        for rc in range(max(0, c - 2), min(w, c + 3)):
            ri = rr * w + rc
            if ri < qi:
                pr, pc = s[ri, 0] + r - rr, s[ri, 1] + c - rc
                if 0 <= pr < A_h and 0 <= pc < A_w:
                    cand.append((A_h * im[ri] + pr) * A_w + pc)
    qs.append(q)
    us.append(((As[np.array(cand)] - q) ** 2).sum(axis=1).min() if cand else np.inf)
Q, Uc = np.array(qs), np.array(us)
an2 = (X ** 2).sum(axis=1)
Qc = Q - mu


def nn_rows(Qs):
    """exact-enough NN row and distance of each query (centred dot products, chunked)"""
    rows, ds = [], []
    for i in range(0, len(Qs), 64):
        qc = Qs[i:i + 64] - mu
        d = an2[None] - 2 * qc @ X.T
        j = d.argmin(axis=1)
        rows.append(j)
        ds.append(np.maximum(0.0, d[np.arange(len(j)), j] + (qc ** 2).sum(axis=1)))
    return np.concatenate(rows), np.concatenate(ds)


_, dnn = nn_rows(Q)
# candidate sources: the causal neighbours' NN rows shifted, and the coarse level's pick upsampled
nbq, nbkey = [], {}
for r in range(r_lo, r_hi + 1):
    c = step - 3 * r
    qi = r * w + c
    for rr in range(max(0, r - 2), r + 1):
        for rc in range(max(0, c - 2), min(w, c + 3)):
            ri = rr * w + rc
            if ri < qi and ri not in nbkey:
                nbkey[ri] = len(nbq)
                nbq.append(O.query_feature(Bf, Bp_sm, O.state_at(Bp_f, job.Bp_init[level], ri), rr, rc, w))
nb_rows, _ = nn_rows(np.array(nbq))
hc, wc = job.B_pyr[level - 1].shape[:2]
Ahc, Awc = job.A_pyr[level - 1].shape[:2]
sc, imc = z['s_%d' % (level - 1)].astype(np.int64), z['im_%d' % (level - 1)].astype(np.int64)
Uns, Uup, Uold = [], [], []
for k, r in enumerate(range(r_lo, r_hi + 1)):
    c = step - 3 * r
    qi = r * w + c
    best = Uc[k]
    # the candidates of every neighbour but the two merged one step earlier ((r, c-1), (r-1, c+2)):
    # what a gather could evaluate before that step's merges end
    old_best = np.inf
    for rr in range(max(0, r - 2), r + 1):
        for rc in range(max(0, c - 2), min(w, c + 3)):
            ri = rr * w + rc
            if ri < qi and (rr, rc) not in ((r, c - 1), (r - 1, c + 2)):
                pr, pc = s[ri, 0] + r - rr, s[ri, 1] + c - rc
                if 0 <= pr < A_h and 0 <= pc < A_w:
                    old_best = min(old_best, ((As[(A_h * im[ri] + pr) * A_w + pc] - Q[k]) ** 2).sum())
                row = int(nb_rows[nbkey[ri]])
                img, rem = divmod(row, A_h * A_w)
                pr, pc = divmod(rem, A_w)
                pr, pc = pr + r - rr, pc + c - rc
                if 0 <= pr < A_h and 0 <= pc < A_w:
                    old_best = min(old_best, ((As[(img * A_h + pr) * A_w + pc] - Q[k]) ** 2).sum())
    Uold.append(old_best)
    for rr in range(max(0, r - 2), r + 1):
        for rc in range(max(0, c - 2), min(w, c + 3)):
            ri = rr * w + rc
            if ri < qi:
                row = int(nb_rows[nbkey[ri]])
                img, rem = divmod(row, A_h * A_w)
                pr, pc = divmod(rem, A_w)
                pr, pc = pr + r - rr, pc + c - rc
                if 0 <= pr < A_h and 0 <= pc < A_w:
                    best = min(best, ((As[(img * A_h + pr) * A_w + pc] - Q[k]) ** 2).sum())
    Uns.append(best)
    ci = min(r // 2, hc - 1) * wc + min(c // 2, wc - 1)
    pr, pc = 2 * sc[ci, 0] + r % 2, 2 * sc[ci, 1] + c % 2
    up = ((As[(imc[ci] * A_h + pr) * A_w + pc] - Q[k]) ** 2).sum() if pr < A_h and pc < A_w else np.inf
    Uup.append(min(best, up))
Uns, Uup, Uold = np.array(Uns), np.array(Uup), np.array(Uold)
Qp = Qc @ U_.T
M = len(Q)
qorder = np.argsort(morton([quant(Qp[:, i], lo[i], hi[i], bits) for i in range(npc)], bits), kind='stable')
print('%s level %d step %d: %d queries; U / NN median %.3f (p10 %.3f, p90 %.3f)' % (
    cfg, level, step, M, np.median(Uc / dnn), np.percentile(Uc / dnn, 10), np.percentile(Uc / dnn, 90)))
for label, Ub in (('+ neighbours NN shifted', Uns), ('+ coarse pick upsampled', Uup),
                  ('nbr sets w/o step-t px', Uold)):
    print('  %-24s U / NN median %.3f (p10 %.3f, p90 %.3f)' % (label, np.median(Ub / dnn), np.percentile(Ub / dnn, 10),
                                                              np.percentile(Ub / dnn, 90)))
for label, Ub in (('U = coherence (today)', Uc), ('U = + nbr NN shifted', Uns), ('U = + coarse upsampled', Uup), ('U = w/o step-t pixels', Uold), ('U = 1.2 NN', 1.2 * dnn), ('U = 1.07 NN', 1.07 * dnn),
                  ('U = NN', dnn)):
    need = np.zeros(nt, dtype=bool)
    pairs = 0
    nqt = -(-M // 32)
    for j in range(nqt):
        ids = qorder[j * 32:(j + 1) * 32]
        d = np.maximum(0, np.maximum(blo[None] - Qp[ids, None], Qp[ids, None] - bhi[None]))
        tn = ((d ** 2).sum(axis=2) <= Ub[ids, None]).any(axis=0)
        pairs += tn.sum()
        need |= tn
    print('  %-24s DB tiles loaded %.4f   pairs %.4f' % (label, need.mean(), pairs / (nqt * nt)))
