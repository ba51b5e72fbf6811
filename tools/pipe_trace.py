"""Level pipelining trace check: from a rocprofv3 kernel trace of a pipelined
`bench.py` run, the finest level's chain of the LAST job on its own stream: wall time from its
first gather to its last merge, kernel time by kind, the time between its kernels, and the other
streams' kernel time inside that window (the coarser levels overlapping it).
  python3 tools/pipe_trace.py <run_kernel_trace.csv> [steps = 4093]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
T = int(sys.argv[2]) if len(sys.argv) > 2 else 4093
for r in rows:
    r['s'], r['e'] = int(r['Start_Timestamp']), int(r['End_Timestamp'])
rows.sort(key=lambda r: r['s'])
sk = 'Stream_Id' if 'Stream_Id' in rows[0] else 'Queue_Id'
fin = [r for r in rows if 'k3h_prune' in r['Kernel_Name']]
st = fin[-1][sk]
mine = [r for r in rows if r[sk] == st]
pr = [i for i, r in enumerate(mine) if 'k3h_prune' in r['Kernel_Name']]
# the last finest-level instance that other streams overlap (a pipelined job; bench.py's
# roofline pass at the end runs the levels on one stream)
other_end = max((r['e'] for r in rows if r[sk] != st and r[sk] != rows[0][sk]), default=0)
k = len(pr) // T
while k > 1 and mine[pr[(k - 1) * T]]['s'] > other_end:
    k -= 1
first = max(pr[(k - 1) * T] - 1, 0)   # the step-0 gather precedes the level's first scan
last = pr[k * T - 1] + 1               # its last merge follows the last scan
KINDS = ('k_gather_query_p', 'k3h_prune', 'k_merge_level', 'k_merge_gather')
lev = [r for r in mine[first:last + 1] if any(kd in r['Kernel_Name'] for kd in KINDS)]
t0, t1 = lev[0]['s'], lev[-1]['e']
by = defaultdict(float)
for r in lev:
    by[r['Kernel_Name'].split('(')[0][:40]] += (r['e'] - r['s']) / 1e6
busy = sum(by.values())
print('finest level on stream %s: %d kernels, wall %.1f ms, kernels %.1f ms, between kernels %.1f ms (%.2f us per kernel)'
      % (st, len(lev), (t1 - t0) / 1e6, busy, (t1 - t0) / 1e6 - busy, ((t1 - t0) / 1e6 - busy) * 1e3 / max(len(lev) - 1, 1)))
for k, v in sorted(by.items(), key=lambda kv: -kv[1]):
    n = sum(1 for r in lev if r['Kernel_Name'].split('(')[0][:40] == k)
    print('  %-40s %5d x %6.1f us = %6.1f ms' % (k, n, v * 1e3 / n, v))
# the job: its kernels on every (queue, stream) since the previous job's last finest-level merge
prev_end = max((r['e'] for r in mine[:first] if 'k_merge' in r['Kernel_Name']), default=0)
job = [r for r in rows if r['s'] > prev_end and r['s'] < t1 + 1]
j0 = min(r['s'] for r in job)
print('job: first kernel %.1f ms before the finest level, last one %.1f ms after its start'
      % ((t0 - j0) / 1e6, (max(r['e'] for r in job) - t0) / 1e6))
span = defaultdict(lambda: [None, None, 0, 0.0, 0.0])
for r in job:
    key = (r['Queue_Id'], r['Stream_Id'])
    sp = span[key]
    sp[0] = r['s'] if sp[0] is None else min(sp[0], r['s'])
    sp[1] = r['e'] if sp[1] is None else max(sp[1], r['e'])
    sp[2] += 1
    sp[3] += (r['e'] - r['s']) / 1e6
    if r['e'] > t0 and r['s'] < t1 and r[sk] != st:
        sp[4] += (min(r['e'], t1) - max(r['s'], t0)) / 1e6
for key, sp in sorted(span.items()):
    print('  queue %s stream %s: %5d kernels %.1f ms, from %+.1f to %+.1f ms (finest level = 0); %.1f ms inside its window'
          % (key[0], key[1], sp[2], sp[3], (sp[0] - t0) / 1e6, (sp[1] - t0) / 1e6, sp[4]))
