#!/bin/bash
# option nn_bound: exactness (pruned-level GPU tests) and the cfg3 / cfg4 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_debug.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap', round(r.get('chain_gap_us_timed',0),2), 'pairs', round(r.get('pairs_frac',0),3), 'corr', round(r.get('pairs_corrected_frac',0),3), 'tiles', round(r.get('tiles_passing_frac',0),3), 'fallbacks', d['stats']['fallbacks'])"; }
for i in 1 2; do
  for v in "c3:--steps 10" "c3nb0:--steps 10 --nn-bound 0" "c4:--config cfg4 --steps 3" "c4nb0:--config cfg4 --steps 3 --nn-bound 0"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 300 python -u bench.py --warmup 1 --no-cpu-baseline $a > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "bench $n failed"; tail -20 $O/${n}_$i.err; exit 1; }
    summ $O/${n}_$i.json $n
  done
done
echo ALL-OK
