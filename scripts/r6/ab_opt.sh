#!/bin/bash
# round 6: same-box A/B of bench.py options on the product library.
#   scripts/r6/ab_opt.sh OUT TESTS "A-args" "B-args" [config]
# TESTS: "full" = the whole -m gpu suite, "core" = prune / debug / pipeline / batch, "none"
# cfg3 pipelined twice each (A, B, A, B), then sequential once each; output under gpurun_out/OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$1; T=$2; A=$3; B=$4; CFG=${5:-cfg3}; mkdir -p $O
case $T in
  full) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }; tail -1 $O/pytest.log;;
  core) timeout -k 10 600 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_debug.py tests/test_gpu_pipeline.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }; tail -1 $O/pytest.log;;
esac
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('$n', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms parity', d.get('parity'), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap s>m', round(r.get('chain_gap_scan_merge_us_timed',0),2), 'gap m>s', round(r.get('chain_gap_merge_scan_us_timed',0),2), 'win', round(r.get('chain_window_ms_timed',0),1))"
}
run A $A || exit 1
run B $B || exit 1
run A2 $A || exit 1
run B2 $B || exit 1
run A_seq $A --pipeline 0 || exit 1
run B_seq $B --pipeline 0 || exit 1
echo ALL-OK
