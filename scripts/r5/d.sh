#!/bin/bash
# round 5: PMC counters of the pruned scan, v24 (two-pass) against v22, cfg3 sequential; the
# gap microbenchmark with the real kernels' argument size and written bytes; the rank-count sort
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${R5_OUT:-r5d}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_debug.py -x -q --timeout 200 --timeout-method thread -k "24 or 25" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
pass() {  # name variant counters...
  local name=$1 v=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex k3h_prune3 --output-format csv \
      -d "$O/$name" -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --time-stride 0 --pipeline 0 --k3p-variant $v \
      > "$O/$name.log" 2>&1 || { echo "pass $name failed rc=$?"; tail -5 "$O/$name.log"; return 1; }
}
for v in 24 22; do
pass a_v$v $v SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA || exit 1
pass b_v$v $v SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES || exit 1
pass f_v$v $v FETCH_SIZE || exit 1
done
python3 tools/pmc_ratio.py $O > $O/pmc_ratio.txt 2>&1; cat $O/pmc_ratio.txt
rm -rf $O/a_v* $O/b_v* $O/f_v*   # the raw CSVs (tens of MB): the summary above is what is kept
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('$n', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms parity', d.get('parity'), 'frac_timed', round(r.get('frac_timed',0),3), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'spread', round(r.get('k3_start_spread_us_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap', round(r.get('chain_gap_us_timed',0),2), 'win', round(r.get('chain_window_ms_timed',0),1))"
}
run v24 --k3p-variant 24 || exit 1
run v22 || exit 1
run v24_b --k3p-variant 24 || exit 1
run c4_v25 --config cfg4 --k3p-variant 25 || exit 1
IA_LIBIA=$PWD/image-analogies-python_amd/libia_probe16.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --pipeline 0 --k3p-variant 24 > $O/probe_v24.json 2> $O/probe_v24.err || { echo "probe failed"; tail -20 $O/probe_v24.err; exit 1; }
grep K3P_PROBE $O/probe_v24.err | tail -5
echo ALL-OK
