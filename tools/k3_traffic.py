"""HBM bytes per K3 launch from tools/pmc_k3.sh output (FETCH_SIZE / WRITE_SIZE passes), with
the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of wide
coalesced streaming reads (x2); WRITE_SIZE is exact.  Averaged over every K3 dispatch of the
profiled bench step, like bench.py's roofline.achieved.  Writes profiles/k3_traffic.json.
  python3 tools/k3_traffic.py <pmc_dir> [out.json]"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, '*', 'run_counter_collection.csv')):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] == counter and 'k3h' in r['Kernel_Name']:
                vals[r['Dispatch_Id']] = vals.get(r['Dispatch_Id'], 0.0) + float(r['Counter_Value'])
    return list(vals.values())


d = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                         'profiles', 'k3_traffic.json')
fetch, write = per_dispatch(d, 'FETCH_SIZE'), per_dispatch(d, 'WRITE_SIZE')
rd = 2.0 * 1024 * sum(fetch) / len(fetch)
wr = 1024.0 * sum(write) / len(write)
res = {'hbm_bytes_per_launch': rd + wr, 'read_bytes_per_launch': rd, 'write_bytes_per_launch': wr,
       'launches': len(fetch), 'source': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), '
       'FETCH_SIZE x2 per MI355X_MICROARCH.md gfx950 note; mean over all K3 dispatches of one cfg3 step'}
json.dump(res, open(out, 'w'), indent=1)
print(json.dumps(res))
