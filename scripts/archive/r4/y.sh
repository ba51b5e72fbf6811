#!/bin/bash
# pipelined jobs: the coarser levels' merge + gather fused (default) or separate
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4y; mkdir -p $O
summ() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M px/s', 'k3p', round(r.get('k3_us_per_launch_timed',0) or 0,2), 'spread', round(r.get('k3_start_spread_us_timed',0) or 0,2), 'merge', round(r.get('merge_us_per_launch_timed',0) or 0,2), 'gap', round(r.get('chain_gap_us_timed',0) or 0,2), 'window', round(r.get('chain_window_ms_timed',0) or 0,1))"; }
for i in 1 2; do
  for v in "c3:--steps 10" "c3cf0:--steps 10 --coarse-fuse-gather 0" "c4:--config cfg4 --steps 3" "c4cf0:--config cfg4 --steps 3 --coarse-fuse-gather 0"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 300 python -u bench.py --warmup 1 --no-cpu-baseline $a > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "bench $n failed"; tail -20 $O/${n}_$i.err; exit 1; }
    summ $O/${n}_$i.json $n
  done
done
echo ALL-OK
