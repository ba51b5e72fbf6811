#!/bin/bash
# round 5: the host-side knobs re-checked on the final kernels (same box, two passes each)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5s; mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('$n', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms parity', d.get('parity'), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'spread', round(r.get('k3_start_spread_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap s>m', round(r.get('chain_gap_scan_merge_us_timed',0),2), 'm>s', round(r.get('chain_gap_merge_scan_us_timed',0),2), 'win', round(r.get('chain_window_ms_timed',0),1))"
}
for pass in 1 2; do
run def$pass || exit 1
run fu$pass --fuse-unpruned 1 || exit 1
run cfg0_$pass --coarse-fuse-gather 0 || exit 1
run ctx3_$pass --pipe-ctx 3 || exit 1
run ctx5_$pass --pipe-ctx 5 || exit 1
run pmr_$pass --prune-min-rows 524288 || exit 1
done
echo ALL-OK
