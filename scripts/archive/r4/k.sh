#!/bin/bash
# with nn_bound on: the hi-only DB stream (k3p_variant 22 / 23), pruning cfg4's 1024^2 B level (512^2 A), k3p_lockstep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_prune.py::test_nn_bound_is_exact_and_tighter tests/test_gpu_prune.py::test_pruned_equals_unpruned tests/test_gpu_batch.py::test_batched_g256_wide_steps_match_reference -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap', round(r.get('chain_gap_us_timed',0),2), 'pairs', round(r.get('pairs_frac',0),3), 'corr', round(r.get('pairs_corrected_frac',0),3), 'tiles', round(r.get('tiles_passing_frac',0),3), 'fallbacks', d['stats']['fallbacks'])"; }
for i in 1 2; do
  for v in "c3:--steps 10" "c3v22:--steps 10 --k3p-variant 22" "c4:--config cfg4 --steps 3" "c4v22:--config cfg4 --steps 3 --k3p-variant 22" "c4p512:--config cfg4 --steps 3 --prune-min-rows 262144" "c4ls:--config cfg4 --steps 3 --k3p-lockstep 1" "c4ls22:--config cfg4 --steps 3 --k3p-lockstep 1 --k3p-variant 22"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 300 python -u bench.py --warmup 1 --no-cpu-baseline $a > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "bench $n failed"; tail -20 $O/${n}_$i.err; exit 1; }
    summ $O/${n}_$i.json $n
  done
done
echo ALL-OK
