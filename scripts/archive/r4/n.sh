#!/bin/bash
# new defaults (nn_bound, k3p_variant 22, cfg4 prunes the 512^2 A level): the whole GPU suite,
# (after the chained-wave budget) cfg3 / cfg4 lines (cfg4 also with fuse_sort 2), cfg5 with and without pruning its 512^2 finest
# levels, and the fused merge + gather phase stamps of the PROBE=8 build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
summ() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'k3p', round(r.get('k3_us_per_launch_timed',0) or 0,2), 'merge', round(r.get('merge_us_per_launch_timed',0) or 0,2), 'gap', round(r.get('chain_gap_us_timed',0) or 0,2), 'pairs', round(r.get('pairs_frac',0) or 0,3), 'tiles', round(r.get('tiles_passing_frac',0) or 0,3), 'fallbacks', d['stats']['fallbacks'])"; }
for i in 1 2; do
  vs=("c3:--steps 10" "c4:--config cfg4 --steps 3" "c4fs2:--config cfg4 --steps 3 --fuse-sort 2")
  [ $i = 1 ] && vs+=("c5:--config cfg5 --steps 2" "c5p512:--config cfg5 --steps 2 --prune-min-rows 262144" "c3seq:--steps 5 --pipeline 0" "c3seqp512:--steps 5 --pipeline 0 --prune-min-rows 262144")
  for v in "${vs[@]}"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 300 python -u bench.py --warmup 1 --no-cpu-baseline $a > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "bench $n failed"; tail -20 $O/${n}_$i.err; exit 1; }
    summ $O/${n}_$i.json $n
  done
done
for p in 0 1; do  # fused merge + gather phase stamps (diagnostic build PROBE=8)
  IA_LIBIA=image-analogies-python_amd/libia_probe8.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --pipeline $p > $O/probe_p$p.txt 2> $O/probe_p$p.err || { echo "probe $p failed"; tail -20 $O/probe_p$p.err; exit 1; }
  grep -c GSTAMP $O/probe_p$p.txt
done
echo ALL-OK
