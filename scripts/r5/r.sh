#!/bin/bash
# round 5: the v24 ring refilled as soon as a slot is read (three tiles in flight, libia.so)
# against the committed kernels (libia_base.so, IA_K3P_REFILL=0); exactness first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_debug.py tests/test_gpu_batch.py tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, lib, args...
  local n=$1 lib=$2; shift 2
  IA_LIBIA=$PWD/image-analogies-python_amd/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('$n', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms parity', d.get('parity'), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'spread', round(r.get('k3_start_spread_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap s>m', round(r.get('chain_gap_scan_merge_us_timed',0),2), 'm>s', round(r.get('chain_gap_merge_scan_us_timed',0),2), 'win', round(r.get('chain_window_ms_timed',0),1))"
}
run new libia.so || exit 1
run base libia_base.so || exit 1
run new_b libia.so || exit 1
run base_b libia_base.so || exit 1
run new_seq libia.so --pipeline 0 || exit 1
run base_seq libia_base.so --pipeline 0 || exit 1
run c4_new libia.so --config cfg4 || exit 1
run c4_base libia_base.so --config cfg4 || exit 1
echo ALL-OK
