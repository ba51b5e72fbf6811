#!/bin/bash
# same-box A/B of (library, bench flags) pairs: ab_runs.sh OUT "name|lib.so|flags" ... (two passes, 10 steps;
# cfg3 unless the flags name another --config)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
for pass in 1 2; do
  for spec in "$@"; do
    IFS='|' read -r n lib flags <<< "$spec"
    IA_LIBIA=$PWD/image-analogies-python_amd/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline $flags > $O/${n}_$pass.json 2> $O/${n}_$pass.err || { echo "bench $n failed"; tail -20 $O/${n}_$pass.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/${n}_$pass.json')); r=d['roofline']; s=d['stats']
print('%-10s' % '$n', $pass, round(d['value']/1e6,3), 'M px/s parity', d.get('parity'), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'spread', round(r.get('k3_start_spread_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gaps', round(r.get('chain_gap_scan_merge_us_timed',0),2), round(r.get('chain_gap_merge_scan_us_timed',0),2), 'stolen', s.get('stolen_tiles'), 'tiles', s.get('dist_tiles'), 'fb', s.get('fallbacks'))"
  done
done
echo ALL-OK
