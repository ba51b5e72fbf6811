#!/bin/bash
# GPU suite, then chain gaps (kernel-stamped) of the finest level across modes + prefetch A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
summ() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap', round(r.get('chain_gap_us_timed',0),2), 'window', round(r.get('chain_window_ms_timed',0),1), 'fallbacks', d['stats']['fallbacks'])"; }
for v in "base:" "nopf:--prefetch-next 0" "seq:--pipeline 0" "seqnopf:--pipeline 0 --prefetch-next 0" "p512:--prune-min-rows 262144" "base2:" "nopf2:--prefetch-next 0"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 200 python -u bench.py --steps 8 --warmup 1 --no-cpu-baseline $a > $O/${n}.json 2> $O/${n}.err || { echo "bench $n failed"; tail -20 $O/${n}.err; exit 1; }
  summ $O/${n}.json $n
done
echo ALL-OK
