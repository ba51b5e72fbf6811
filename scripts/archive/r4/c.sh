#!/bin/bash
# same-box A/B of the pipelined job: default vs pruning the 512^2 level too; plus the
# sequential (one level at a time) stamped kernel times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4c; mkdir -p $O
summ() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'k3p launches', r.get('k3_launches_timed'), 'fallbacks', d['stats']['fallbacks'])"; }
for i in 1 2; do
  for v in "base:--fuse-sort 0" "p512:--fuse-sort 0 --prune-min-rows 262144" "seq:--fuse-sort 0 --pipeline 0"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 200 python -u bench.py --steps 8 --warmup 1 --no-cpu-baseline $a > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "bench $n failed"; tail -20 $O/${n}_$i.err; exit 1; }
    summ $O/${n}_$i.json $n
  done
done
echo ALL-OK
