#!/bin/bash
# cfg3 on the final kernels: the in-gather sort (fuse_sort 1) against the in-scan sort
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4z; mkdir -p $O
summ() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M px/s', 'k3p', round(r.get('k3_us_per_launch_timed',0) or 0,2), 'wg', round(r.get('k3_wg_us_timed',0) or 0,2), 'merge', round(r.get('merge_us_per_launch_timed',0) or 0,2), 'gap', round(r.get('chain_gap_us_timed',0) or 0,2))"; }
for i in 1 2; do
  for v in "c3:--steps 10" "c3fs1:--steps 10 --fuse-sort 1"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 300 python -u bench.py --warmup 1 --no-cpu-baseline $a > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "bench $n failed"; tail -20 $O/${n}_$i.err; exit 1; }
    summ $O/${n}_$i.json $n
  done
done
echo ALL-OK
