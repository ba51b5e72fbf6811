#!/bin/bash
# work stealing: the stealing test, the prune / debug / pipeline suites, then the bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-steal}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_prune.py -k "stealing" -s > $O/t_steal.log 2>&1 || { echo "steal test failed"; tail -30 $O/t_steal.log; exit 1; }
grep -E "stolen|passed|failed" $O/t_steal.log | tail -4
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_prune.py tests/test_gpu_debug.py tests/test_gpu_pipeline.py tests/test_gpu_parity.py > $O/t_suites.log 2>&1 || { echo "suites failed"; tail -30 $O/t_suites.log; exit 1; }
tail -1 $O/t_suites.log
for pass in 1 2; do
  for v in 0 1; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --steal $v > $O/s${v}_$pass.json 2> $O/s${v}_$pass.err || { echo "bench steal $v failed"; tail -20 $O/s${v}_$pass.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/s${v}_$pass.json')); r=d['roofline']
print('steal $v pass $pass', round(d['value']/1e6,3), 'M px/s parity', d.get('parity'), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'spread', round(r.get('k3_start_spread_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gaps', round(r.get('chain_gap_scan_merge_us_timed',0),2), round(r.get('chain_gap_merge_scan_us_timed',0),2), 'stolen', d['stats'].get('stolen_tiles'), 'fb', d['stats'].get('fallbacks'))"
  done
done
echo ALL-OK
