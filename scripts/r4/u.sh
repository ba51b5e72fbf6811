#!/bin/bash
# end-of-round check: the whole GPU suite, smoke, and the default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${R4U_OUT:-r4u}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print(round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'steps', d['steps'], 'frac_timed', round(r['frac_timed'],3), 'k3p', round(r['k3_us_per_launch_timed'],2), 'wg', round(r['k3_wg_us_timed'],2), 'spread', round(r['k3_start_spread_us_timed'],2))"
echo ALL-OK
