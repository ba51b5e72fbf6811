#!/bin/bash
# round 5: k3p_variant 24 as the default - the whole GPU suite + smoke; the kernel-boundary
# microbenchmark with the scan's DB stream (L2s full of clean lines at each boundary); v25 with
# the gathers' sort against v24; the PMC wait ratio of the default scan
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${R5_OUT:-r5f}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for m in 0 2 6; do
  timeout -k 10 120 ./tools/gap_micro 1000 $m > $O/gap_micro_m$m.txt 2>&1 || { echo "gap_micro $m failed"; cat $O/gap_micro_m$m.txt; exit 1; }
  echo "== gap_micro mode $m"; cat $O/gap_micro_m$m.txt
done
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('$n', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms parity', d.get('parity'), 'frac_timed', round(r.get('frac_timed',0),3), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'spread', round(r.get('k3_start_spread_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap', round(r.get('chain_gap_us_timed',0),2), 'win', round(r.get('chain_window_ms_timed',0),1))"
}
run v24 || exit 1
run v25fs --k3p-variant 25 --fuse-sort 1 || exit 1
run v24_b || exit 1
run v25fs_b --k3p-variant 25 --fuse-sort 1 || exit 1
run v24_seq --pipeline 0 || exit 1
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex k3h_prune3 --output-format csv \
      -d "$O/$name" -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --time-stride 0 --pipeline 0 \
      > "$O/$name.log" 2>&1 || { echo "pass $name failed rc=$?"; tail -5 "$O/$name.log"; return 1; }
}
pass a_v24 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA || exit 1
pass b_v24 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES || exit 1
pass f_v24 FETCH_SIZE || exit 1
python3 tools/pmc_ratio.py $O > $O/pmc_ratio.txt 2>&1; cat $O/pmc_ratio.txt
rm -rf $O/a_v24 $O/b_v24 $O/f_v24
echo ALL-OK
