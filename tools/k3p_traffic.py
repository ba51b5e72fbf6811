"""HBM bytes per launch of the pruned scan (k3h_prune3) from tools/pmc_k3p.sh output, with the
gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE reports half the bytes of wide coalesced
streaming reads: x2; WRITE_SIZE is exact).  hbm_bytes_per_launch = the mean over the finest
level's dispatches (the last <finest_dispatches> of a sequential bench step, --pipeline 0: the
level bench.py's roofline describes); plateau_* = their middle half.  Writes
profiles/k3p_traffic_<config>.json and prints the SQ counters of the plateau dispatches.
  python3 tools/k3p_traffic.py <pmc_dir> [out.json] [config] [finest_dispatches] [kernel]
(cfg3: 4093 = the 1024^2 level's steps; cfg4: 16378 = 8189 steps of 2 launches each; kernel:
the dominant kernel's name substring, k3h_prune3 by default, k3h_scan for cfg5's unpruned scans)"""
import csv
import glob
import json
import os
import sys

CONFIG = sys.argv[3] if len(sys.argv) > 3 else 'cfg3'
LEVEL9_STEPS = int(sys.argv[4]) if len(sys.argv) > 4 else 4093  # finest level's pruned dispatches
KERNEL = sys.argv[5] if len(sys.argv) > 5 else 'k3h_prune3'


def per_dispatch(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] == counter and KERNEL in r['Kernel_Name']:
                k = int(r['Dispatch_Id'])
                vals[k] = vals.get(k, 0.0) + float(r['Counter_Value'])
    return [vals[k] for k in sorted(vals)]


def plateau(v):
    v = v[-LEVEL9_STEPS:]
    return v[len(v) // 4: 3 * len(v) // 4]


d = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                         'profiles', 'k3p_traffic_%s.json' % CONFIG)
fa, wa = per_dispatch(os.path.join(d, 'fetch'), 'FETCH_SIZE'), per_dispatch(os.path.join(d, 'write'), 'WRITE_SIZE')
fp, wp = plateau(fa), plateau(wa)
# the finest level's dispatches (the last <finest_dispatches> of a sequential step: bench.py's
# roofline describes the pruned level with the largest DB, ia_stats.prune_rows)
ff, wf = fa[-LEVEL9_STEPS:], wa[-LEVEL9_STEPS:]
rd = 2.0 * 1024 * sum(ff) / len(ff)
wr = 1024.0 * sum(wf) / len(wf)
rdp = 2.0 * 1024 * sum(fp) / len(fp)
wrp = 1024.0 * sum(wp) / len(wp)
res = {'hbm_bytes_per_launch': rd + wr, 'read_bytes_per_launch': rd, 'write_bytes_per_launch': wr,
       'launches': len(ff), 'all_pruned_launches': len(fa), 'plateau_hbm_bytes_per_launch': rdp + wrp, 'plateau_read_bytes_per_launch': rdp,
       'plateau_write_bytes_per_launch': wrp, 'plateau_launches': len(fp), 'kernel': KERNEL,
       'source': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes; KB units), FETCH_SIZE x2 per '
                 'MI355X_MICROARCH.md gfx950 note (Infinity-Cache hits are counted); mean over the finest level\'s '
                 'dispatches of the kernel in one sequential %s bench step (the level bench.py\'s roofline describes); '
                 'plateau_* = their middle half' % CONFIG, 'config': CONFIG}
sq = {}
for c in ('SQ_WAVE_CYCLES', 'SQ_BUSY_CYCLES', 'SQ_INSTS_VALU', 'SQ_INSTS_MFMA', 'SQ_INSTS_LDS',
          'SQ_VALU_MFMA_BUSY_CYCLES', 'SQ_LDS_BANK_CONFLICT', 'GRBM_GUI_ACTIVE'):
    v = plateau(per_dispatch(os.path.join(d, 'sq'), c))
    if v:
        sq[c] = sum(v) / len(v)
res['sq_plateau_per_launch'] = sq
json.dump(res, open(out, 'w'), indent=1)
print(json.dumps(res, indent=1))
