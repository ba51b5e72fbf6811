"""Per-level, per-kernel device time from a rocprofv3 --kernel-trace CSV of bench.py.
Levels are delimited by the per-level k_part_means launch.  Usage:
  python3 tools/trace_breakdown.py <run_kernel_trace.csv> [job_index]"""
import collections
import csv
import re
import sys


def short(name):
    for k in ('k_part_means_fold', 'k3h_prune', 'k_gather_query_p', 'k3h_scan', 'k3h_dist', 'k3_dist', 'k_merge_level',
              'k_merge_xchg', 'k_query_sort', 'k_gather_query_h', 'k_gather_query', 'k_part_means',
              'k_db_build_h', 'k_db_build', 'k_absmax', 'k_reduce_stats', 'k_finish_level', 'k_step_fused'):
        if k in name:
            return k
    return re.sub(r'\(.*', '', name)[:30]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
job = int(sys.argv[2]) if len(sys.argv) > 2 else 0
levels, cur, spans = [], None, []
for r in rows:
    k = short(r['Kernel_Name'])
    if k == 'k_part_means':
        cur = collections.defaultdict(lambda: [0, 0.0])
        levels.append(cur)
        spans.append([int(r['Start_Timestamp']), int(r['End_Timestamp'])])
    if cur is None:
        continue
    spans[-1][1] = max(spans[-1][1], int(r['End_Timestamp']))
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    cur[k][0] += 1
    cur[k][1] += d
    cur[k].append(d)
per_job = 9
sel = levels[job * per_job:(job + 1) * per_job] if len(levels) >= per_job else levels
ssp = spans[job * per_job:(job + 1) * per_job] if len(levels) >= per_job else spans
tot = collections.defaultdict(float)
for i, lv in enumerate(sel):
    s = sum(v[1] for v in lv.values())
    wall = (ssp[i][1] - ssp[i][0]) / 1e6
    print('level %d: %.1f ms (wall %.1f ms: %.1f ms between kernels)  ' % (i + 1, s / 1e3, wall, wall - s / 1e3) + '  '.join('%s %d x %.1fus=%.1fms' % (k, v[0], v[1] / max(v[0], 1), v[1] / 1e3)
                                                          for k, v in sorted(lv.items(), key=lambda x: -x[1][1]) if v[1] > 100))
    for k, v in lv.items():
        tot[k] += v[1]
# duration percentiles of the finest level's per-step kernels (median vs mean: the tail's share)
if sel:
    lv = sel[-1]
    for k, v in sorted(lv.items(), key=lambda x: -x[1][1]):
        ds = sorted(v[2:])
        if len(ds) >= 100:
            q = lambda f: ds[min(len(ds) - 1, int(f * len(ds)))]
            print('  %s finest level: mean %.1f p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f us (tail above p90: %.1f ms)'
                  % (k, v[1] / v[0], q(.1), q(.5), q(.9), q(.99), ds[-1], sum(x - q(.9) for x in ds if x > q(.9)) / 1e3))
print('total %.1f ms: ' % (sum(tot.values()) / 1e3) + ', '.join('%s %.1f' % (k, v / 1e3) for k, v in sorted(tot.items(), key=lambda x: -x[1])))
