#!/bin/bash
# round 5: the stream's need test on 8-query sub-boxes (IA_K3P_SUBBOX, libia.so) against the
# per-query test (libia_pq.so); exactness first; the two chain boundaries split
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${R5_OUT:-r5g}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_debug.py tests/test_gpu_batch.py tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, lib, args...
  local n=$1 lib=$2; shift 2
  IA_LIBIA=$PWD/image-analogies-python_amd/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('$n', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms parity', d.get('parity'), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'spread', round(r.get('k3_start_spread_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap s>m', round(r.get('chain_gap_scan_merge_us_timed',0),2), 'm>s', round(r.get('chain_gap_merge_scan_us_timed',0),2), 'win', round(r.get('chain_window_ms_timed',0),1), 'pairs', r.get('pairs_frac'), 'passing', r.get('tiles_passing_frac'))"
}
run sb libia.so || exit 1
run pq libia_pq.so || exit 1
run sb_b libia.so || exit 1
run pq_b libia_pq.so || exit 1
run sb_seq libia.so --pipeline 0 || exit 1
run pq_seq libia_pq.so --pipeline 0 || exit 1
run c4_sb libia.so --config cfg4 || exit 1
run c4_pq libia_pq.so --config cfg4 || exit 1
IA_LIBIA=$PWD/image-analogies-python_amd/libia_probe16.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --pipeline 0 > $O/probe_sb.json 2> $O/probe_sb.err || { echo "probe failed"; tail -20 $O/probe_sb.err; exit 1; }
grep K3P_PROBE $O/probe_sb.err | tail -5
echo ALL-OK
