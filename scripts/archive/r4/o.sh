#!/bin/bash
# option prefetch_rows (LDS-DMA of the next query's older U' candidate rows): exactness, cfg3 / cfg4 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_prune.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'k3p', round(r.get('k3_us_per_launch_timed',0) or 0,2), 'merge', round(r.get('merge_us_per_launch_timed',0) or 0,2), 'gap', round(r.get('chain_gap_us_timed',0) or 0,2), 'pairs', round(r.get('pairs_frac',0) or 0,3), 'tiles', round(r.get('tiles_passing_frac',0) or 0,3), 'fallbacks', d['stats']['fallbacks'])"; }
for i in 1 2; do
  for v in "c3:--steps 10" "c3pr:--steps 10 --prefetch-rows 1" "c4:--config cfg4 --steps 3" "c4pr:--config cfg4 --steps 3 --prefetch-rows 1"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 300 python -u bench.py --warmup 1 --no-cpu-baseline $a > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "bench $n failed"; tail -20 $O/${n}_$i.err; exit 1; }
    summ $O/${n}_$i.json $n
  done
done
echo ALL-OK
