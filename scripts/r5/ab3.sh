#!/bin/bash
# round 5: two experimental builds ($1, $2) against the product library, cfg3 pipelined, twice
# each in turn (no tests: timing split of an experiment already tested exact); gpurun_out/$3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$3; mkdir -p $O
run() {  # name, lib, args...
  local n=$1 lib=$2; shift 2
  IA_LIBIA=$PWD/image-analogies-python_amd/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('$n', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms parity', d.get('parity'), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'win', round(r.get('chain_window_ms_timed',0),1))"
}
for r in a b; do
  run x1_$r $1 || exit 1
  run x2_$r $2 || exit 1
  run base_$r libia.so || exit 1
done
echo ALL-OK
