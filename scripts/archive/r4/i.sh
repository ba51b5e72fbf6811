#!/bin/bash
# cfg4 (683-query steps): the gathers' sort (fuse_sort) replaces the K2s launch of every step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4i; mkdir -p $O
summ() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap', round(r.get('chain_gap_us_timed',0),2), 'window', round(r.get('chain_window_ms_timed',0),1), 'fallbacks', d['stats']['fallbacks'])"; }
for i in 1 2; do
  for v in "c4:--config cfg4" "c4fs:--config cfg4 --fuse-sort 1"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline $a > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "bench $n failed"; tail -20 $O/${n}_$i.err; exit 1; }
    summ $O/${n}_$i.json $n
  done
done
echo ALL-OK
