"""DESIGN.md §7 cost model of the DB-sharded path from a rocprofv3 kernel trace of
`bench.py --shard-emulate W [--shard-jobs J]` (all W shards of every large level run back to back
on one GPU; with J jobs every scan and merge covers all J jobs' queries: bench.py's N > 1 shard
mode at J = W, whose weak-scaling efficiency is the W = 1 single-job time / the modelled time).
Per wavefront step of each level the trace holds: the query gather (K2), the W shard scans
(K3h / K3p; + the query sort K2s on wide steps) and the W exchange merges (k_merge_xchg: W - 1
publishing launches, then the finishing one) - or, on levels too small to shard, one scan and
one merge.  On W real ranks each rank runs K2, ITS shard's scan and one finishing merge, so a
step costs
    K2 + max over shards (scan) + finishing merge + x
with x the exchange latency (an xGMI store + the peers' polling: a parameter, default 3 us).
Owner-computes steps (exchange = 2: per step W gathers, W sorts, W scans, W merges, one per
emulated rank) cost max(gather) + max(sort) + max(scan) + max(merge) + 2 x.
Printed: measured kernel time per level (this one-GPU emulation) and the modelled per-rank time
on W GPUs, per level and for the job; speedup and efficiency against the W = 1 model.
  python3 tools/shard_model.py <run_kernel_trace.csv> <W> [x_us] [baseline_job_ms] [w1_model.txt]"""
import csv
import re
import sys

# optional 5th argument: the W = 1 run's model output; in owner-computes runs a level with no
# sharded step runs only the rank's own job there, i.e. takes the one-job time
BASE_LV = {}
if len(sys.argv) > 5:
    for ln in open(sys.argv[5]):
        mm = re.match(r'level (\d+): .* modelled per rank ([\d.]+) ms', ln)
        if mm:
            BASE_LV[int(mm.group(1))] = float(mm.group(2)) * 1e3
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
W = int(sys.argv[2])
XLAT = float(sys.argv[3]) if len(sys.argv) > 3 else 3.0
base = float(sys.argv[4]) if len(sys.argv) > 4 else None


def kind(name):
    if 'k_part_means' in name and 'fold' not in name:
        return 'level'
    if 'k_gather_query' in name:
        return 'gather'
    if 'k3h_' in name or 'k3_dist' in name:
        return 'scan'
    if 'k_query_sort' in name:
        return 'sort'
    if 'k_merge_xchg' in name or 'k_merge_level' in name or 'k_finish_level' in name or 'k_merge_gather' in name:
        return 'merge'
    return 'other'


levels = []   # per level: list of steps, each {gathers[], sorts[], scans[], merges[]}
step = None
last = None
for r in rows:
    k = kind(r['Kernel_Name'])
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    if k == 'level':
        levels.append({'steps': [], 'other': 0.0})
        step = last = None
        continue
    if not levels:
        continue
    lv = levels[-1]
    # a step starts with its gather(s), or - when the previous step's fused merge + gather
    # (k_merge_gather) ran them - with its sort / scan right after a merge
    if (k == 'gather' and last not in ('gather', 'sort')) or (k in ('sort', 'scan') and last in ('merge', None)):
        step = {'gathers': [], 'sorts': [], 'scans': [], 'merges': [], 'owner': False}
        lv['steps'].append(step)
    # owner-computes steps: one fused merge per owner (k_merge_level<CH, true, ...> or k_merge_gather);
    # the RCCL exchange's per-shard merges are k_merge_level<CH, false, ...>
    if k == 'merge' and step is not None and ('k_merge_gather' in r['Kernel_Name'] or
                                              re.search(r'k_merge_level<\d+, true', r['Kernel_Name'])):
        step['nown'] = step.get('nown', 0) + 1
    if step is None or k in ('other', 'level'):
        lv['other'] += d
    else:
        step[k + 's'].append(d)
    last = k

# the bench's timed step is the last job of the trace: its levels are the last L - 1 entries
L = 9 if len(levels) >= 9 else len(levels)
sel = levels[-L:]
tot_meas = tot_model = 0.0
for i, lv in enumerate(sel):
    meas = model = 0.0
    sharded = 0
    for st in lv['steps']:
        meas += sum(st['gathers']) + sum(st['sorts']) + sum(st['scans']) + sum(st['merges'])
        nsh = len(st['merges'])
        sharded += nsh > 1
        if len(st['gathers']) > 1 or st.get('nown', 0) > 1:
            # owner-computes step (exchange = 2): every emulated owner's gather, sort and merge
            # are its rank's own launches; each rank pays the slowest of each plus its shard's
            # scan and two exchange latencies (sorted queries out, records back)
            model += max(st['gathers'] or [0.0]) + max(st['sorts'] or [0.0]) + max(st['scans'] or [0.0]) + \
                max(st['merges']) + 2 * XLAT
            continue
        # scans of one shard are consecutive launches (several query blocks of an unpruned or
        # unsharded level run one after the other): a rank pays its shard's sum
        sc = st['scans']
        per = len(sc) // nsh if nsh > 1 and len(sc) % nsh == 0 else len(sc)
        grp = [sum(sc[i:i + per]) for i in range(0, len(sc), per)] if sc else [0.0]
        model += sum(st['gathers']) + sum(st['sorts']) + max(grp) + (st['merges'][-1] if st['merges'] else 0.0) + \
            (XLAT if nsh > 1 else 0.0)
    meas += lv['other']
    model += lv['other']
    owner = any(len(st['gathers']) > 1 or st.get('nown', 0) > 1 for l2 in sel for st in l2['steps'])
    if owner and sharded == 0 and (i + 1) in BASE_LV:
        model = BASE_LV[i + 1]
    tot_meas += meas
    tot_model += model
    print('level %d: %d steps (%d sharded %d ways): emulated %.1f ms, modelled per rank %.1f ms'
          % (i + 1, len(lv['steps']), sharded, W, meas / 1e3, model / 1e3))
print('job: emulated kernels %.1f ms on one GPU; modelled %.1f ms per rank on %d GPUs (exchange latency %.1f us/step)'
      % (tot_meas / 1e3, tot_model / 1e3, W, XLAT))
if base:
    if any(len(st['gathers']) > 1 or st.get('nown', 0) > 1 for lv in sel for st in lv['steps']):
        # owner computes: W jobs on W ranks (weak scaling): efficiency = one job alone / per-rank time
        print('weak scaling vs %.1f ms for one job on one GPU: efficiency %.0f %% (%d jobs in %.1f ms on %d GPUs)'
              % (base, 100 * base / (tot_model / 1e3), W, tot_model / 1e3, W))
    else:
        print('speedup vs %.1f ms: %.2fx, efficiency %.0f %%' % (base, base / (tot_model / 1e3), 100 * base / (tot_model / 1e3) / W))
