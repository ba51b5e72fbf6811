"""Teacher-force a GPU-synthesised cfg3 state offline (SURVEY §7 hard part 2).

The GPU box runs `python tools/dump_state.py gpurun_out/cfg3_state.npz 1024 1 2 ... 9` (every
level's final B', s, im).  Here, the job's host inputs are rebuilt deterministically
(ia_amd.synth.make_job, same seeds) and the oracle (oracle/ia_oracle.py decide_pixel: exact fp64
NN in numpy's order, best_coherence_match, compute_distance in the BLAS order, the kappa rule)
re-decides sampled pixels on the GPU's own state: B' final for raster-earlier pixels, initial
for the rest, s / im final.  Every decision must match except documented near-ties (NN relative
gap < 1e-5, kappa relative margin < 1e-12).  Test infrastructure: uses the oracle.

  python tools/teacher_force.py <state.npz> <out.json> [total_pixels] [workers] [finest_min]

finest_min: at least this many pixels on the finest dumped level.  States written by
tools/dump_state.py with a config name (cfg3, cfg4) rebuild that config's job.
"""
import json
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

_G = {}


def _job(cfg):
    import ia_amd  # noqa: F401
    from ia_amd import synth
    return synth.make_job(**(dict(size=int(cfg)) if cfg.isdigit() else synth.CONFIGS[cfg][0]))


def rebuild_bp(job, z, level):
    """B' of a synthesised level from its source maps: B'[p] = A'_im[p][s[p]] (the merge's
    writeback), checked against the sha1 of the GPU's own B' bytes (tools/dump_state.py)"""
    import hashlib
    s = z['s_%d' % level].astype(np.int64)
    im = z['im_%d' % level].astype(np.int64)
    Ap = np.stack([p[level] for p in job.Ap_pyr_list])
    bp = Ap[im, s[:, 0], s[:, 1]].reshape(job.B_pyr[level].shape[:2])
    if hashlib.sha1(np.ascontiguousarray(bp).tobytes()).digest() != z['bpsha_%d' % level].tobytes():
        raise SystemExit("level %d: B' rebuilt from s / im differs from the GPU's B'" % level)
    return bp


def _init(path, cfg):
    _G['job'] = _job(cfg)
    z = np.load(path)
    _G['z'] = {k: z[k] for k in z.files}
    for l in sorted({int(k.split('_')[1]) for k in z.files if k.startswith('s_')}):
        if 'Bp_%d' % l not in _G['z']:
            _G['z']['Bp_%d' % l] = rebuild_bp(_G['job'], z, l)
    _G['db'] = {}


def _decide(args):
    from oracle import ia_oracle as O
    level, pix = args
    job, z = _G['job'], _G['z']
    if level not in _G['db']:
        _G['db'] = {level: (O.build_db(job.A_pyr, job.Ap_pyr_list, level), O.feature_array(job.B_pyr, level, True))}
    As, Bf = _G['db'][level]
    h, w = job.B_pyr[level].shape[:2]
    A_h, A_w = job.A_pyr[level].shape[:2]
    Bp_l, Bp_c = z['Bp_%d' % level], z['Bp_%d' % (level - 1)]
    s, im = z['s_%d' % level].astype(np.int64), z['im_%d' % level].astype(np.int64)
    out = []
    for qi in pix:
        r, c = divmod(int(qi), w)
        d = O.decide_pixel(As, Bf, Bp_c, Bp_l, job.Bp_init[level], s, im, A_h, A_w, level, job.L, job.k, job.weights,
                           r, c)
        (pr, pc), img = d['choice']
        ok = (pr, pc, img) == (s[qi, 0], s[qi, 1], im[qi])
        out.append((level, int(qi), bool(ok), float(d['app_gap']), float(d.get('kappa_gap', 1.0))))
    return out


def main():
    path, out_json = sys.argv[1], sys.argv[2]
    total = int(sys.argv[3]) if len(sys.argv) > 3 else 5000
    workers = int(sys.argv[4]) if len(sys.argv) > 4 else 7
    finest_min = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    z = np.load(path)
    cfg = str(z['config']) if 'config' in z.files else str(int(z['size']))
    levels = [int(l) for l in z['levels']]
    job = _job(cfg)
    # pixels per level: proportional to sqrt(N) (every level gets a share; the 1024^2 level most)
    npx = {l: int(np.prod(job.B_pyr[l].shape[:2])) for l in levels}
    wts = {l: np.sqrt(npx[l]) for l in levels}
    tot_w = sum(wts.values())
    tasks = []
    for l in levels:
        n = min(npx[l], max(20, int(round(total * wts[l] / tot_w)), finest_min if l == max(levels) else 0))
        h, w = job.B_pyr[l].shape[:2]
        rs = np.random.RandomState(1000 + l)
        pix = np.unique(np.concatenate([rs.choice(npx[l], n, replace=False), [0, 1, w - 1, w, npx[l] - 1]]))
        for chunk in np.array_split(pix, max(1, len(pix) // 25)):
            tasks.append((l, chunk))
    t0 = time.time()
    with Pool(workers, initializer=_init, initargs=(path, cfg)) as pool:
        res = [r for part in pool.imap_unordered(_decide, tasks) for r in part]
    per_level = {}
    mism = []
    for level, qi, ok, gap, kgap in res:
        d = per_level.setdefault(level, {'pixels': 0, 'mismatches': 0, 'near_ties_nn': 0, 'near_ties_kappa': 0})
        d['pixels'] += 1
        d['near_ties_nn'] += gap < 1e-5
        d['near_ties_kappa'] += kgap < 1e-12
        if not ok:
            d['mismatches'] += 1
            mism.append({'level': level, 'pixel': qi, 'nn_rel_gap': gap, 'kappa_rel_margin': kgap,
                         'documented_near_tie': gap < 1e-5 or kgap < 1e-12})
    summary = {'state': os.path.basename(path), 'job': 'synth.make_job(%s)' % cfg,
               'pixels_checked': len(res), 'mismatches': len(mism),
               'undocumented_mismatches': sum(1 for m in mism if not m['documented_near_tie']),
               'per_level': {str(k): per_level[k] for k in sorted(per_level)}, 'mismatch_list': mism,
               'near_tie_rule': 'NN relative gap < 1e-5 or kappa relative margin < 1e-12',
               'seconds': time.time() - t0, 'workers': workers}
    with open(out_json, 'w') as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: summary[k] for k in ('pixels_checked', 'mismatches', 'undocumented_mismatches', 'seconds')}))


if __name__ == '__main__':
    main()
