#!/bin/bash
# round 5: (1) kernel boundaries with the first stamp after the kernel arguments, kernel
# arguments in device memory or not; (2) exactness of the chunk-major records + sub-box coarse
# need test (libia.so); (3) A/B: libia.so against query-major records (libia_qm.so) and against
# the tile-box coarse test with query-major records (libia_pq.so); (4) the sort-phase probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${R5_OUT:-r5i}; mkdir -p $O
for m in 8; do
  for dk in 0 1; do
    HIP_FORCE_DEV_KERNARG=$dk timeout -k 10 120 ./tools/gap_micro 1000 $m > $O/gap_micro_m${m}_dk$dk.txt 2>&1 || { echo "gap_micro failed"; cat $O/gap_micro_m${m}_dk$dk.txt; exit 1; }
    echo "== gap_micro mode $m HIP_FORCE_DEV_KERNARG=$dk"; head -3 $O/gap_micro_m${m}_dk$dk.txt
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_prune.py tests/test_gpu_debug.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, lib, args...
  local n=$1 lib=$2; shift 2
  IA_LIBIA=$PWD/image-analogies-python_amd/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('$n', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms parity', d.get('parity'), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'spread', round(r.get('k3_start_spread_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap s>m', round(r.get('chain_gap_scan_merge_us_timed',0),2), 'm>s', round(r.get('chain_gap_merge_scan_us_timed',0),2), 'win', round(r.get('chain_window_ms_timed',0),1), 'pairs', round(r.get('pairs_frac',0),4), 'passing', round(r.get('tiles_passing_frac',0),4))"
}
run new libia.so || exit 1
run qm libia_qm.so || exit 1
run pq libia_pq.so || exit 1
run new_b libia.so || exit 1
run qm_b libia_qm.so || exit 1
run pq_b libia_pq.so || exit 1
run new_seq libia.so --pipeline 0 || exit 1
run qm_seq libia_qm.so --pipeline 0 || exit 1
HIP_FORCE_DEV_KERNARG=1 run new_dk libia.so || exit 1
HIP_FORCE_DEV_KERNARG=1 run new_dk_seq libia.so --pipeline 0 || exit 1
IA_LIBIA=$PWD/image-analogies-python_amd/libia_probe16.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --pipeline 0 > $O/probe.json 2> $O/probe.err || { echo "probe failed"; tail -20 $O/probe.err; exit 1; }
grep K3P_PROBE $O/probe.err | tail -7
echo ALL-OK
