#!/bin/bash
# round 5: v24 with the tile counter back in the stream + a shared pass list; exactness, A/B, probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${R5_OUT:-r5e}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_debug.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread -k "24 or 25" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('$n', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms parity', d.get('parity'), 'frac_timed', round(r.get('frac_timed',0),3), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'spread', round(r.get('k3_start_spread_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap', round(r.get('chain_gap_us_timed',0),2), 'win', round(r.get('chain_window_ms_timed',0),1))"
}
run v24 --k3p-variant 24 || exit 1
run v22 || exit 1
run v24_b --k3p-variant 24 || exit 1
run c4_v24 --config cfg4 --k3p-variant 24 || exit 1
run c5_v24 --config cfg5 --k3p-variant 24 || exit 1
run c5_v22 --config cfg5 || exit 1
IA_LIBIA=$PWD/image-analogies-python_amd/libia_probe16.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --pipeline 0 --k3p-variant 24 > $O/probe_v24.json 2> $O/probe_v24.err || { echo "probe failed"; tail -20 $O/probe_v24.err; exit 1; }
grep K3P_PROBE $O/probe_v24.err | tail -5
echo ALL-OK
