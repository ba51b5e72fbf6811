#!/bin/bash
# cfg3 pipelined: pruning the 256^2 (and 128^2) levels too
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4p; mkdir -p $O
summ() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'k3p', round(r.get('k3_us_per_launch_timed',0) or 0,2), 'merge', round(r.get('merge_us_per_launch_timed',0) or 0,2), 'gap', round(r.get('chain_gap_us_timed',0) or 0,2), 'window', round(r.get('chain_window_ms_timed',0) or 0,1), 'fallbacks', d['stats']['fallbacks'])"; }
for i in 1 2; do
  for v in "c3:--steps 10" "c3p256:--steps 10 --prune-min-rows 65536" "c3p128:--steps 10 --prune-min-rows 16384" "c4p256:--config cfg4 --steps 3 --prune-min-rows 65536"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 300 python -u bench.py --warmup 1 --no-cpu-baseline $a > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "bench $n failed"; tail -20 $O/${n}_$i.err; exit 1; }
    summ $O/${n}_$i.json $n
  done
done
echo ALL-OK
