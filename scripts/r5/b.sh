#!/bin/bash
# round 5: the two-pass pruned scan (k3p_variant 24 / 25) - exactness first, then a same-box A/B
# against round 4's library (libia_base.so, v22) and the K3p phase probe of the round-4 kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${R5_OUT:-r5b}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_prune.py -x -q --timeout 200 --timeout-method thread -k "24 or 25" > $O/pytest_prune.log 2>&1 || { echo "prune tests failed"; tail -30 $O/pytest_prune.log; exit 1; }
tail -1 $O/pytest_prune.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_debug.py -x -q --timeout 200 --timeout-method thread -k "v24 or v25" > $O/pytest_debug.log 2>&1 || { echo "debug tests failed"; tail -30 $O/pytest_debug.log; exit 1; }
tail -1 $O/pytest_debug.log
run() {  # name, lib, args...
  local n=$1 lib=$2; shift 2
  IA_LIBIA=$PWD/image-analogies-python_amd/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('$n', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'frac_timed', round(r.get('frac_timed',0),3), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'spread', round(r.get('k3_start_spread_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap', round(r.get('chain_gap_us_timed',0),2), 'win', round(r.get('chain_window_ms_timed',0),1), 'pass_tiles', round(r.get('tiles_passing_frac',0),3))"
}
run base_v22 libia_base.so || exit 1
run new_v22 libia.so || exit 1
run new_v24 libia.so --k3p-variant 24 || exit 1
run base_v22_seq libia_base.so --pipeline 0 || exit 1
run new_v24_seq libia.so --pipeline 0 --k3p-variant 24 || exit 1
run new_v24_b libia.so --k3p-variant 24 || exit 1
run base_v22_b libia_base.so || exit 1
for v in 22 24; do
IA_LIBIA=$PWD/image-analogies-python_amd/libia_probe16.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --pipeline 0 --k3p-variant $v > $O/probe_v$v.json 2> $O/probe_v$v.err || { echo "probe failed"; tail -20 $O/probe_v$v.err; exit 1; }
echo "== probe v$v"; grep K3P_PROBE $O/probe_v$v.err | tail -5
done
timeout -k 10 120 ./tools/gap_micro 2000 > $O/gap_micro.txt 2>&1 || { echo "gap_micro failed"; cat $O/gap_micro.txt; exit 1; }
cat $O/gap_micro.txt
echo ALL-OK
