#!/bin/bash
# where a K3p launch's time goes: workgroup start spread vs mean workgroup duration vs tail,
# sequential and pipelined cfg3, and cfg4; plus the stats-struct CPU/GPU agreement (prune tests)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4r; mkdir -p $O
summ() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M px/s', 'k3p', round(r.get('k3_us_per_launch_timed',0) or 0,2), 'wg', round(r.get('k3_wg_us_timed',0) or 0,2), 'start_spread', round(r.get('k3_start_spread_us_timed',0) or 0,2), 'merge', round(r.get('merge_us_per_launch_timed',0) or 0,2), 'gap', round(r.get('chain_gap_us_timed',0) or 0,2))"; }
for v in "c3:--steps 10" "c3seq:--steps 5 --pipeline 0" "c4:--config cfg4 --steps 3"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py --warmup 1 --no-cpu-baseline $a > $O/${n}.json 2> $O/${n}.err || { echo "bench $n failed"; tail -20 $O/${n}.err; exit 1; }
  summ $O/${n}.json $n
done
echo ALL-OK
