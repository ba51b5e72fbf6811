#!/bin/bash
# round-6 final evidence, part B1: the scan's PMC wait ratio (sequential cfg3); part B2 is final_b2.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6final}; mkdir -p $O
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex k3h_prune3 --output-format csv \
      -d "$O/$name" -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --time-stride 0 --pipeline 0 \
      > "$O/$name.log" 2>&1 || { echo "pass $name failed rc=$?"; tail -5 "$O/$name.log"; return 1; }
}
pass a_v24 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA || exit 1
pass b_v24 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES || exit 1
python3 tools/pmc_ratio.py $O > $O/pmc_ratio.txt 2>&1; cat $O/pmc_ratio.txt
rm -rf $O/a_v24 $O/b_v24
echo ALL-OK
