#!/bin/bash
# round 5: a same-box A/B of an experimental build (image-analogies-python_amd/$1) against the
# product library (libia.so): exactness of the experiment first, then cfg3 pipelined twice each
# and sequential once each; output under gpurun_out/$2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
X=$1; O=gpurun_out/$2; mkdir -p $O
IA_LIBIA=$PWD/image-analogies-python_amd/$X timeout -k 10 600 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_debug.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, lib, args...
  local n=$1 lib=$2; shift 2
  IA_LIBIA=$PWD/image-analogies-python_amd/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('$n', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms parity', d.get('parity'), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'win', round(r.get('chain_window_ms_timed',0),1))"
}
run exp $X || exit 1
run base libia.so || exit 1
run exp_b $X || exit 1
run base_b libia.so || exit 1
run exp_seq $X --pipeline 0 || exit 1
run base_seq libia.so --pipeline 0 || exit 1
echo ALL-OK
