"""Medians of the fused merge + gather phase stamps of a PROBE=8 build (stderr lines STAMP / GSTAMP,
one sampled wave per 256 steps; s_memtime cycles) for the widest level (or bw=<w> in argv[2])."""
import re
import sys
from collections import defaultdict

import numpy as np

lines = open(sys.argv[1]).read().splitlines()
want = int(sys.argv[2]) if len(sys.argv) > 2 else None
rows = defaultdict(lambda: defaultdict(list))
for ln in lines:
    if not (ln.startswith('STAMP') or ln.startswith('GSTAMP') or ln.startswith('ESTAMP')):
        continue
    kv = dict(re.findall(r'(\w[\w+]*)=(\d+)', ln))
    bw = int(kv['bw'])
    tag = 'G' if ln.startswith('GSTAMP') else 'E' if ln.startswith('ESTAMP') else 'M'
    for k, v in kv.items():
        if k not in ('bw', 't', 'M'):
            rows[bw][tag + ':' + k].append(int(v))
bw = want or max(rows)
names = {'M:d1': 'records round', 'M:d2': 'candidate placement', 'M:d3': 'fp64 rows round', 'M:d4': 'reductions',
         'M:d5': 'certification', 'M:d6': 'kappa', 'M:d7': 'writes', 'G:merge': 'merge (whole)',
         'G:handoff_wait': 'wait for the row above', 'G:gather': 'gather (whole)', 'G:feat+frag': '  features + fragments',
         'G:sums': '  wave sums', 'G:urow': "  U' rows round", 'G:rec': '  pruning record',
         'E:pre': 'early gather: features, sums', 'E:part': "  U' partials (rows landed)",
         'E:handoff': '  wait for the row above', 'E:late': '  late slot + U\' min', 'E:rec': '  pruning record'}
print('bw=%d: %d merge samples, %d gather samples' % (bw, len(rows[bw]['M:d1']), len(rows[bw]['G:merge'])))
for k, n in names.items():
    if rows[bw][k]:
        a = np.array(rows[bw][k])
        print('  %-28s median %7.0f  p90 %7.0f' % (n, np.median(a), np.percentile(a, 90)))
