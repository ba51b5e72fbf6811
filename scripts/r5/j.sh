#!/bin/bash
# round 5: the in-kernel query sort as per-wave runs + a rank merge (libia.so) against the
# 512-lane bitonic network (libia_bn.so); exactness first (every in-kernel-sort path: prune,
# debug, batch, shard), then a same-box A/B and the phase probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${R5_OUT:-r5j}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_debug.py tests/test_gpu_batch.py tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, lib, args...
  local n=$1 lib=$2; shift 2
  IA_LIBIA=$PWD/image-analogies-python_amd/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('$n', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms parity', d.get('parity'), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'spread', round(r.get('k3_start_spread_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap s>m', round(r.get('chain_gap_scan_merge_us_timed',0),2), 'm>s', round(r.get('chain_gap_merge_scan_us_timed',0),2), 'win', round(r.get('chain_window_ms_timed',0),1))"
}
run ws libia.so || exit 1
run bn libia_bn.so || exit 1
run ws_b libia.so || exit 1
run bn_b libia_bn.so || exit 1
run ws_seq libia.so --pipeline 0 || exit 1
run bn_seq libia_bn.so --pipeline 0 || exit 1


IA_LIBIA=$PWD/image-analogies-python_amd/libia_probe16.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --pipeline 0 > $O/probe.json 2> $O/probe.err || { echo "probe failed"; tail -20 $O/probe.err; exit 1; }
grep K3P_PROBE $O/probe.err | tail -7
echo ALL-OK
