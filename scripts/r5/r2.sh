#!/bin/bash
# round 5: the v24 ring refilled after the next-tile search (libia_r2.so, IA_K3P_REFILL=2)
# against the committed kernels (libia_base.so, IA_K3P_REFILL=0); exactness first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5r2; mkdir -p $O
IA_LIBIA=$PWD/image-analogies-python_amd/libia_r2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_debug.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, lib, args...
  local n=$1 lib=$2; shift 2
  IA_LIBIA=$PWD/image-analogies-python_amd/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('$n', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms parity', d.get('parity'), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'win', round(r.get('chain_window_ms_timed',0),1))"
}
run r2 libia_r2.so || exit 1
run base libia_base.so || exit 1
run r2_b libia_r2.so || exit 1
run base_b libia_base.so || exit 1
echo ALL-OK
