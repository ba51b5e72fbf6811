#!/bin/bash
# option k3p_pool (dynamic hand-out of the last tiles of every K3p chunk): exactness, then the cfg3 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4x; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_prune.py -x -q -k "pool" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M px/s', 'k3p', round(r.get('k3_us_per_launch_timed',0) or 0,2), 'wg', round(r.get('k3_wg_us_timed',0) or 0,2), 'spread', round(r.get('k3_start_spread_us_timed',0) or 0,2), 'merge', round(r.get('merge_us_per_launch_timed',0) or 0,2), 'fallbacks', d['stats']['fallbacks'])"; }
for i in 1 2; do
  for v in "c3:--steps 10" "c3p5:--steps 10 --k3p-pool 5" "c3p10:--steps 10 --k3p-pool 10" "c3p20:--steps 10 --k3p-pool 20"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 300 python -u bench.py --warmup 1 --no-cpu-baseline $a > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "bench $n failed"; tail -20 $O/${n}_$i.err; exit 1; }
    summ $O/${n}_$i.json $n
  done
done
echo ALL-OK
