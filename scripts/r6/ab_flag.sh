#!/bin/bash
# same-box A/B of one bench.py flag: ab_flag.sh OUT FLAG VALUE... (two passes each, cfg3, 10 steps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$1; F=$2; shift 2; mkdir -p $O
for pass in 1 2; do
  for v in "$@"; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline $F $v > $O/v${v}_$pass.json 2> $O/v${v}_$pass.err || { echo "bench $F $v failed"; tail -20 $O/v${v}_$pass.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/v${v}_$pass.json')); r=d['roofline']
print('$F $v pass $pass', round(d['value']/1e6,3), 'M px/s parity', d.get('parity'), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'spread', round(r.get('k3_start_spread_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gaps', round(r.get('chain_gap_scan_merge_us_timed',0),2), round(r.get('chain_gap_merge_scan_us_timed',0),2), 'window', round(r.get('chain_window_ms_timed',0),1))"
  done
done
echo ALL-OK
