#!/bin/bash
# K3p (v22) wait anatomy from SQ counters: the share of wave cycles spent waiting (cfg3, sequential)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4w; mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-include-regex k3h_prune3 --output-format csv -d $O/wait -o run -- python3 bench.py --config cfg3 --steps 1 --warmup 0 --no-cpu-baseline --time-stride 0 --pipeline 0 > $O/wait.log 2>&1 || { echo "pmc failed rc=$?"; tail -5 $O/wait.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/r4w/wait/**/run_counter_collection.csv', recursive=True)
rows = list(csv.DictReader(open(f[0])))
agg = collections.defaultdict(list)
for r in rows:
    if 'k3h_prune3' in r.get('Kernel_Name', '') and 'Li11E' in r.get('Kernel_Name', ''):
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
m = {k: sum(v) / len(v) for k, v in agg.items()}
print({k: round(v) for k, v in m.items()})
if m.get('SQ_WAVE_CYCLES'):
    print('wait_any / wave_cycles = %.3f, wait_inst_any / wave_cycles = %.3f' % (m.get('SQ_WAIT_ANY', 0) / m['SQ_WAVE_CYCLES'], m.get('SQ_WAIT_INST_ANY', 0) / m['SQ_WAVE_CYCLES']))
PY
rm -rf $O/wait/*/*/*.csv.tmp 2>/dev/null
echo ALL-OK
