#!/bin/bash
# round 6: same-box A/B of experimental libraries against the product library (libia.so):
#   scripts/r6/ab_libs.sh OUT "bench args" lib1.so [lib2.so ...]
# cfg3 (or the config in the bench args) pipelined, rounds of base then each lib, twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$1; ARGS=$2; shift 2; mkdir -p $O
run() {  # name, lib
  local n=$1 lib=$2
  IA_LIBIA=$PWD/image-analogies-python_amd/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline $ARGS > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('%-14s' % '$n', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms parity', d.get('parity'), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gaps', round(r.get('chain_gap_scan_merge_us_timed',0),2), round(r.get('chain_gap_merge_scan_us_timed',0),2), 'tpass', round(r.get('tiles_passing_frac',0),4), 'pairs', round(r.get('pairs_frac',0),4))"
}
for pass in 1 2; do
  run base_$pass libia.so || exit 1
  for L in "$@"; do run ${L%.so}_$pass $L || exit 1; done
done
echo ALL-OK
