#!/bin/bash
# round 5: PMC counters of the pruned scan, v24 (two-pass) against v22, cfg3 sequential; the
# gap microbenchmark with the real kernels' argument size and written bytes; the rank-count sort
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${R5_OUT:-r5d}; mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o "SQ_[A-Z_]*" $O/counters.txt | sort -u | tr '\n' ' ' > $O/sq_counters.txt; head -c 3000 $O/sq_counters.txt; echo
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
python3 tools/pmc_summary.py $O 2>&1 | tail -60 || true
timeout -k 10 120 ./tools/gap_micro 2000 1 > $O/gap_micro_real.txt 2>&1 || { echo "gap_micro failed"; cat $O/gap_micro_real.txt; exit 1; }
cat $O/gap_micro_real.txt
IA_LIBIA=$PWD/image-analogies-python_amd/libia_rank.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --k3p-variant 24 > $O/rank_v24.json 2> $O/rank_v24.err || { echo "rank bench failed"; tail -5 $O/rank_v24.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --k3p-variant 24 > $O/v24.json 2> $O/v24.err || { echo "bench failed"; tail -5 $O/v24.err; exit 1; }
for n in rank_v24 v24; do python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('$n', round(d['value']/1e6,3), 'M px/s parity', d.get('parity'), 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'wg', round(r.get('k3_wg_us_timed',0),2), 'pairs', round(r.get('pairs_frac',0),4))"; done
echo ALL-OK
