#!/usr/bin/env python3
"""Per-dispatch means of rocprofv3 --pmc counters over one kernel instance (default: the pruned
scan's QT = 11 instance, i.e. the 1024^2 plateau steps of cfg3), for every pass directory under
<dir>, and the wait / active ratios of SQ_WAVE_CYCLES.
  python3 tools/pmc_ratio.py <dir> [kernel_substring]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else 'k3h_prune3ILi4ELi11E'
res = collections.defaultdict(dict)
for p in sorted(glob.glob(os.path.join(d, '*'))):
    if not os.path.isdir(p):
        continue
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(p, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r['Kernel_Name']:
                vals[r['Counter_Name']][r['Dispatch_Id']] += float(r['Counter_Value'])
    name = os.path.basename(p)
    var = name.split('_')[-1]
    for c, per in vals.items():
        res[var][c] = sum(per.values()) / max(len(per), 1)
        res[var]['_n'] = len(per)
for var in sorted(res):
    r = res[var]
    print('== %s (%d dispatches)' % (var, r.get('_n', 0)))
    for c in sorted(k for k in r if not k.startswith('_')):
        print('  %-28s %14.0f' % (c, r[c]))
    w = r.get('SQ_WAVE_CYCLES')
    if w:
        for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_LDS',
                  'SQ_ACTIVE_INST_MISC', 'SQ_ACTIVE_INST_SCA'):
            if c in r:
                print('  %-28s %.3f of SQ_WAVE_CYCLES' % (c, r[c] / w))
    if 'FETCH_SIZE' in r:
        print('  HBM read bytes per launch (FETCH_SIZE x 1024 x 2, gfx950): %.1f MB' % (r['FETCH_SIZE'] * 2048 / 1e6))
