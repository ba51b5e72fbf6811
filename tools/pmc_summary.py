"""Summarise rocprofv3 --pmc CSVs (tools/pmc_k3.sh) per kernel name: counter totals per dispatch,
averaged over the dispatches whose grid and kernel name match (e.g. the plateau K3 instance)."""
import collections
import csv
import glob
import os
import sys


def load(d, name_filter):
    rows = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for f in glob.glob(os.path.join(d, '*', 'run_counter_collection.csv')):
        for r in csv.DictReader(open(f)):
            if name_filter not in r['Kernel_Name']:
                continue
            key = (os.path.basename(os.path.dirname(f)), r['Dispatch_Id'])
            rows[key][r['Counter_Name']] += float(r['Counter_Value'])
            names[key] = r['Kernel_Name']
    per = collections.defaultdict(list)
    for (p, _), c in rows.items():
        per[p].append(c)
    out = {}
    for p, lst in per.items():
        for cname in lst[0]:
            out[cname] = sum(x[cname] for x in lst) / len(lst)
        out['_n_' + p] = len(lst)
    return out


if __name__ == '__main__':
    flt = sys.argv[2] if len(sys.argv) > 2 else 'ILi11E'
    c = load(sys.argv[1], flt)
    for k in sorted(c):
        print('%-32s %.4g' % (k, c[k]))
    if 'SQ_WAVE_CYCLES' in c and 'SQ_BUSY_CYCLES' in c:
        print('MFMA busy / (busy cycles*4 SIMD) %.3f' % (c['SQ_VALU_MFMA_BUSY_CYCLES'] / max(1, c['SQ_BUSY_CYCLES'] * 4 * 256)))
